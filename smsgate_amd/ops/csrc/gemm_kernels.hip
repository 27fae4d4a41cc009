// smsgate_amd — fused bf16 MFMA GEMMs for the extractor LM on gfx950.
//
//   C[M, Nout] = EPI( rowscale ⊙ (A[M, K] · W[N, K]ᵀ) )
//
// The decode step of a 576-wide model at M = 256…4096 rows is a chain of small-K
// GEMMs (K = 576 / 1536) whose cost in hipBLASLt is dominated by fixed per-tile
// overhead and by the elementwise kernels around them.  One templated kernel
// absorbs those neighbours:
//
//   NORM   RMSNorm prologue.  The norm weight is folded into W on the host
//          (W' = W·diag(w)), and rsqrt(mean(x²)+eps) of every A row is accumulated
//          from the A tiles the kernel streams anyway and applied to the fp32
//          accumulator in the epilogue — the normalised activation never exists
//          in memory.
//   EPI 0  store bf16.
//   EPI 1  residual add: C = R + bf16(acc) (R may alias C: each element is read
//          and written by the same thread) — the o-proj / down-proj epilogue that
//          updates the residual stream in place.
//   EPI 2  SwiGLU: W rows are interleaved in groups of 16 (16 gate rows, then the
//          16 matching up rows), so one lane holds gate and up of the same output
//          element in two accumulators; C = silu(g)·u with Nout = N / 2.
//   EPI 4  lm_head + schema-FSM masked arg-max: nothing is stored; each row's
//          bf16 logits of this N tile are masked with the row's FSM state and
//          reduced to one (value, index) key, merged across N tiles with a 64-bit
//          atomicMax — the [M, V] logits never reach HBM (sg_gemm_argmax).
//
// Tiling (cdna_hip_programming.md §5): 4 or 8 waves, BM×BN block tile,
// BK = 64, 16×16×32 bf16 MFMAs; A/W tiles staged global → registers → LDS,
// double-buffered with one barrier per K-tile (the global loads of tile k+1 are
// in flight while tile k is multiplied).  LDS rows are 128 B with a 16-byte-chunk
// XOR swizzle (chunk ^ (row & 7)) so the 16 rows a fragment read touches spread
// over all banks.  The epilogue stages the bf16 tile through LDS and writes
// 16-byte row chunks (coalesced), which is also where the residual is read.
// Block → tile mapping is XCD-aware: blocks are dealt round-robin to the 8 XCDs,
// so each XCD is given a contiguous range of tiles (tiles sharing A rows share
// that XCD's L2).
#include <hip/hip_runtime.h>
#include <type_traits>
#include <stdint.h>

namespace {

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef float f32x4 __attribute__((ext_vector_type(4)));

constexpr int BK = 64;  // K elements per tile = 8 chunks of 16 B

// EPI 3 (QKV projection + RoPE + KV-cache write) arguments; unused by other epilogues.
struct RopeArgs {
  const int* pos;       // [M] own-key offset of each token
  const int* slot;      // [M] KV slot of each token
  const float2* cs;     // [max_pos][32] (cos, sin), RoPE position = p0 + pos
  uint16_t* q_out;      // [M][nh][64]
  uint16_t* k_cache;    // [S][nkv][Lmax][64]
  uint16_t* vt_cache;   // [S][nkv][Lmax/8][64][8]
  int nh, nkv, Lmax, p0;
  int hb;  // head index of N column 0 (the v-only launch of cfg 39 starts at nh + nkv)
};

// Row scales computed by the PRODUCER of the activation (NORM 2).  An EPI 1 GEMM
// (o-proj / down-proj: it writes the residual stream) with `ssout` set also writes,
// per N tile, the fp32 sum of squares of each output row's bf16 values:
// ssout[tile_n][row] in a zero-padded [SS_PARTS][ld] image (part-major: a tile's rows
// are one contiguous run, so its partials leave as whole lines — a row-major image
// had every N tile write 4 B into the same 64-B lines, +1 µs per GEMM).
// The next RMSNorm GEMM (NORM 2) prefetches its rows' partials at kernel start — the
// 4 lanes that share an output row read 4 parts each and combine with two shuffles
// (fixed order: deterministic, no atomics) — instead of accumulating x² beside its
// MFMAs, which every N tile and every wave column of the consumer would otherwise
// redo for the same rows.
constexpr int SS_PARTS = 16;  // max N tiles of a producer (hidden <= 16 x BN)
struct NormArgs {
  const float* ssin;  // [SS_PARTS][ld] partial sums of squares of the A rows (NORM 2)
  float* ssout;       // [SS_PARTS][ld] partials of the output rows (EPI 1), or null
  int ld;             // row capacity of the image (>= M)
};

// EPI 4 (lm_head + masked arg-max) arguments.
struct ArgmaxArgs {
  const int* row_state;         // [M] FSM state of each row
  const int* state_mask;        // [S] state -> mask row
  const uint32_t* masks;        // [mask rows][N / 32] allowed-token bits
  unsigned long long* best;     // [M] running max of argmax_key(), zeroed before the launch
  // copy-constrained decoding (optional): a row whose state has copy_kind != 0 is
  // masked with its own row_masks[row] (the schema mask AND its body's copy set,
  // built by sg_copy_masks) instead of the state's mask row
  const int* copy_kind;         // [S] or null
  const uint32_t* row_masks;    // [M][N / 32]
};

// Orderable key: larger bf16 value first, then the SMALLER token index (the tie rule
// of fsm_sample_kernel); -0 is folded into +0 so equal values compare equal.
__device__ __forceinline__ unsigned long long argmax_key(float v, int idx) {
  const uint32_t b = __float_as_uint(v + 0.0f);
  const uint32_t k = (b & 0x80000000u) ? ~b : (b | 0x80000000u);
  return ((unsigned long long)k << 32) | (unsigned long long)(0xFFFFFFFFu - (uint32_t)idx);
}

__device__ __forceinline__ float bf2f(uint32_t v) { return __uint_as_float(v << 16); }
__device__ __forceinline__ uint16_t f2bf(float f) {
  __bf16 b = (__bf16)f;
  return __builtin_bit_cast(uint16_t, b);
}
// x·sigmoid(x) with the hardware reciprocal (v_rcp_f32, ~1 ulp): an IEEE division
// is a ~10-instruction sequence and dominated the SwiGLU epilogue's VALU count
__device__ __forceinline__ float silu(float g) { return g * __builtin_amdgcn_rcpf(1.f + __expf(-g)); }

// ---- staging: async global → LDS DMA (global_load_lds_dwordx4).  One wave
// instruction writes 1 KiB = 8 rows × 128 B lane-linearly (lane l → row l>>3,
// physical chunk l&7), so the XOR swizzle is applied on the SOURCE address:
// physical chunk p of row r holds logical chunk p ^ (r & 7).  No staging
// registers — nothing for the compiler to sink or spill (cdna_hip_programming.md §5).
typedef __attribute__((address_space(3))) void* lds_ptr_t;

// BKT 32 (64-B rows, 4 chunks): one instruction writes 16 rows (lane l -> row l>>2,
// physical chunk l&3) and physical chunk p of row r holds logical chunk
// p ^ ((r >> 1) & 2) -- the XOR that keeps every ds_read_b128 lane group of the
// fragment reads on distinct bank slots with 64-B rows (rows r, r+4, r+8, r+12 share
// banks; they differ in bit 2 or 3 of r)
__device__ __forceinline__ int sw32(int row) { return (row >> 1) & 2; }

template <int ROWS, int NW, int BKT = BK>
__device__ __forceinline__ void issue_tile(const uint16_t* __restrict__ src, int ld, int r0, int rmax, int k0,
                                           uint16_t* dst, int wave, int lane) {
  if constexpr (BKT == 32) {
    static_assert(ROWS % 16 == 0, "16-row pieces");
    constexpr int PIECES = ROWS / 16;
    const int rr = lane >> 2, p = lane & 3;
#pragma unroll
    for (int i = 0; i < (PIECES + NW - 1) / NW; ++i) {
      const int g = PIECES % NW == 0 ? wave + NW * i : min(wave + NW * i, PIECES - 1);
      const int row = 16 * g + rr;
      const int gr = min(r0 + row, rmax);
      const uint16_t* gp = src + (size_t)gr * ld + k0 + ((p ^ sw32(row)) << 3);
      __builtin_amdgcn_global_load_lds((const void*)gp, (lds_ptr_t)(dst + g * 16 * BKT), 16, 0, 0);
    }
  } else {
    static_assert(BKT == 64, "BK 64 or 32");
    static_assert(ROWS % 8 == 0, "8-row pieces");
    constexpr int PIECES = ROWS / 8;
    const int rr = lane >> 3, p = lane & 7;
    // every wave issues the same count (the K loop's counted vmcnt): when the pieces do
    // not divide evenly (96 rows over 8 waves), the spare issues re-load the last piece
    // into its own place (same bytes, same LDS address)
#pragma unroll
    for (int i = 0; i < (PIECES + NW - 1) / NW; ++i) {
      const int g = PIECES % NW == 0 ? wave + NW * i : min(wave + NW * i, PIECES - 1);  // 8-row piece
      const int row = 8 * g + rr;
      const int gr = min(r0 + row, rmax);  // rows past the end re-read the last row (never stored)
      const uint16_t* gp = src + (size_t)gr * ld + k0 + ((p ^ (row & 7)) << 3);
      __builtin_amdgcn_global_load_lds((const void*)gp, (lds_ptr_t)(dst + g * 8 * BK), 16, 0, 0);
    }
  }
}

__device__ __forceinline__ float sumsq_frag(const bf16x8& v, float acc) {
  typedef __bf16 bf16x2 __attribute__((ext_vector_type(2)));
  const uint4 u = __builtin_bit_cast(uint4, v);
  acc = __builtin_amdgcn_fdot2_f32_bf16(__builtin_bit_cast(bf16x2, u.x), __builtin_bit_cast(bf16x2, u.x), acc, false);
  acc = __builtin_amdgcn_fdot2_f32_bf16(__builtin_bit_cast(bf16x2, u.y), __builtin_bit_cast(bf16x2, u.y), acc, false);
  acc = __builtin_amdgcn_fdot2_f32_bf16(__builtin_bit_cast(bf16x2, u.z), __builtin_bit_cast(bf16x2, u.z), acc, false);
  acc = __builtin_amdgcn_fdot2_f32_bf16(__builtin_bit_cast(bf16x2, u.w), __builtin_bit_cast(bf16x2, u.w), acc, false);
  return acc;
}

template <int FM, int FN, int NORM, int BKT = BK>
__device__ __forceinline__ void mma_tile(f32x4 (&acc)[FM][FN], float (&ss)[FM], const uint16_t* as,
                                         const uint16_t* bs, int wm0, int wn0, int lane) {
  auto at = [](int row, int ch) { return row * BKT + ((BKT == 64 ? ch ^ (row & 7) : ch ^ sw32(row)) << 3); };
#pragma unroll
  for (int s = 0; s < BKT / 32; ++s) {
    const int ch = s * 4 + (lane >> 4);
    bf16x8 af[FM], bfr[FN];
#pragma unroll
    for (int j = 0; j < FN; ++j) {
      const int row = wn0 + j * 16 + (lane & 15);
      bfr[j] = *reinterpret_cast<const bf16x8*>(bs + at(row, ch));
    }
#pragma unroll
    for (int i = 0; i < FM; ++i) {
      const int row = wm0 + i * 16 + (lane & 15);
      af[i] = *reinterpret_cast<const bf16x8*>(as + at(row, ch));
    }
#pragma unroll
    for (int i = 0; i < FM; ++i) {
#pragma unroll
      for (int j = 0; j < FN; ++j)
        // C^T tile (W rows x A rows): lane holds C[m = lane & 15][n = 4·(lane>>4) + r],
        // 4 consecutive output columns -> one 8-byte LDS write in the epilogue
        acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bfr[j], af[i], acc[i][j], 0, 0, 0);
      // RMSNorm: the A fragment already holds 8 k-values of row (lane & 15) —
      // accumulate their squares (v_dot2_f32_bf16) in the MFMA shadow
      if constexpr (NORM == 1) ss[i] = sumsq_frag(af[i], ss[i]);
    }
  }
}

// PROBE (timing decomposition only, sg_gemm_probe): 1 = K-loop without MFMAs,
// 2 = K-loop without the global->LDS loads (MFMAs on stale LDS), 3 = as 2 and no
// prologue loads either, 4 = as 3 and no epilogue (nothing stored).
// NORM: 0 none, 1 row scale from x² accumulated beside the MFMAs, 2 row scale from
// the producer's partial sums (NormArgs).
template <int BM, int BN, int WM, int WN, int EPI, int NORM, int ST, int PROBE = 0, int BKT = BK>
__global__ void __launch_bounds__(WM * WN * 64) gemm_fused_kernel(const uint16_t* __restrict__ A, int lda,
                                                         const uint16_t* __restrict__ W,
                                                         uint16_t* C, int ldc, const uint16_t* R, int ldr,
                                                         int M, int N, int K, float eps, int tiles_m,
                                                         int tiles_n, int gm, RopeArgs ra, ArgmaxArgs xa,
                                                         NormArgs na) {
  constexpr int NW = WM * WN, NT = NW * 64;  // waves, threads
  static_assert(NW == 4 || NW == 8, "4 or 8 waves");
  static_assert(EPI != 3 || BN % 64 == 0, "QKV+RoPE epilogue: whole 64-wide heads per N tile");
  constexpr int HT = BN / 64;  // EPI 3: heads per N tile (all q, all k or all v: HT | nh, HT | nkv)
  constexpr int TM = BM / WM, TN = BN / WN;  // wave tile
  constexpr int FM = TM / 16, FN = TN / 16;  // MFMA tiles per wave
  static_assert(FM >= 1 && FN >= 1 && TM % 16 == 0 && TN % 16 == 0, "tile");
  static_assert(EPI != 2 || FN % 2 == 0, "SwiGLU pairs gate/up 16-col groups inside a wave tile");
  constexpr int BNO = EPI == 2 ? BN / 2 : BN;  // output columns of the block
  constexpr int CST = BNO + 8;                // staged C row stride (elements), +16 B pad
  constexpr int TILE = (BM + BN) * BKT;       // one stage (A + B) in elements
  constexpr int RPI = BKT == 64 ? 8 : 16;     // rows per LDS-DMA instruction (1 KiB)
  constexpr int NI = (BM / RPI + NW - 1) / NW + (BN / RPI + NW - 1) / NW;  // glds instructions per stage per wave
  static_assert(ST >= 2 && ST <= 4, "pipeline stages");
  static_assert(BM * CST <= ST * TILE, "C staging fits in the K-loop buffers");
  // EPI 1 with a non-power-of-two chunk count per row (96 / 192-wide tiles) sums the
  // rows' x² partials through a [BM][CPR] fp32 image beside the staged C tile; a 256-row
  // tile needs more than its K-loop buffers for the two (the array grows past them)
  constexpr int CPR1 = BNO / 8;
  constexpr int EPI1_LDS = EPI == 1 && (CPR1 & (CPR1 - 1)) != 0 ? BM * CST + 2 * BM * CPR1 : 0;
  constexpr int SMEM = ST * TILE > EPI1_LDS ? ST * TILE : EPI1_LDS;
  static_assert(SMEM * 2 <= 160 * 1024, "LDS");

  // ONE __shared__ array (a second one makes hipcc wait vmcnt(0) before ds_reads)
  __shared__ __attribute__((aligned(16))) uint16_t smem[SMEM];

  // ---- XCD-aware, bijective tile assignment: the blocks of one XCD (orig % 8)
  // get a contiguous range of tiles, so tiles that share A rows share an L2
  const int T = tiles_m * tiles_n;
  const int orig = blockIdx.x, xcd = orig & 7, q8 = T >> 3, r8 = T & 7;
  const int t = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + (orig >> 3);
  // grouped rasterisation: runs of `gm` M-tiles walk N together, so the tiles in
  // flight on an XCD (~64) cover a compact gm x (64/gm) patch of A rows x W rows
  // that stays L2-resident (row-major order sweeps all of W per M-tile row)
  const int gsz = gm * tiles_n, g = t / gsz, gl = t - g * gsz;
  const int grows = min(gm, tiles_m - g * gm);
  const int m0 = (g * gm + gl % grows) * BM;
  const int n0 = (gl / grows) * BN;

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm0 = (wave / WN) * TM, wn0 = (wave % WN) * TN;

  // NORM 2: the rows' x² partials, loaded before the K loop (consumed in the epilogue;
  // the loop's counted waits retire them with the first tile's DMAs)
  f32x4 ssv[FM];
  if constexpr (NORM == 2) {
#pragma unroll
    for (int i = 0; i < FM; ++i) {
      const int row = min(m0 + wm0 + i * 16 + (lane & 15), M - 1);
      const float* sp = na.ssin + (size_t)((lane >> 4) * 4) * na.ld + row;
#pragma unroll
      for (int e = 0; e < 4; ++e) ssv[i][e] = sp[(size_t)e * na.ld];
    }
  }
  // EPI 1: this thread's residual chunks (R may alias C, but every element is read and
  // written by the same thread).  RPRE_EARLY: loaded before the K loop, their latency
  // hidden behind it but their registers live through it; else issued right after the
  // K loop, in flight while the accumulators are staged through LDS
  constexpr int RIT = EPI == 1 ? (BM * (BN / 8) + NT - 1) / NT : 1;  // (32x96: 1.5 chunks per thread)
  constexpr bool RPRE_EARLY = RIT <= 6;
  uint4 rpre[RIT];
  auto load_rpre = [&]() {
#pragma unroll
    for (int it = 0; it < RIT; ++it) {
      const int q = min(tid + it * NT, BM * (BN / 8) - 1), row = q / (BN / 8), c = q % (BN / 8);
      const int gr = min(m0 + row, M - 1);
      rpre[it] = *reinterpret_cast<const uint4*>(R + (size_t)gr * ldr + n0 + c * 8);
    }
  };
  if constexpr (EPI == 1 && RPRE_EARLY) load_rpre();
  // EPI 3: the tile's token positions / KV slots, likewise loaded before the K loop —
  // q/k heads: the rows of this thread's (row, quarter) items; v heads: row = lane (+64)
  constexpr int QIT = (BM * 4 + NT - 1) / NT, VU = BM > 64 ? 2 : 1;
  constexpr int EPN = EPI == 3 ? (QIT > VU ? QIT : VU) : 1;
  int epos[EPN], eslot[EPN];
  if constexpr (EPI == 3) {
    const int h = (n0 >> 6) + ra.hb;
    if (h < ra.nh + ra.nkv) {
#pragma unroll
      for (int it = 0; it < QIT; ++it) {
        const int gr = min(m0 + ((tid + it * NT) >> 2), M - 1);
        epos[it] = ra.pos[gr];
        eslot[it] = h >= ra.nh ? ra.slot[gr] : 0;
      }
    } else {
#pragma unroll
      for (int u = 0; u < VU; ++u) {
        const int gl = min(m0 + u * 64 + lane, M - 1);
        epos[u] = ra.pos[gl];
        eslot[u] = ra.slot[gl];
      }
    }
  }
  // EPI 4: the FSM state of each of this thread's epilogue rows, likewise (one link of
  // the row_state -> state_mask -> mask-word chain fewer after the K loop)
  constexpr int XIT = EPI == 4 ? (BM * (BN / 8)) / NT : 1;
  int xstate[XIT];
  if constexpr (EPI == 4) {
#pragma unroll
    for (int it = 0; it < XIT; ++it) xstate[it] = xa.row_state[min(m0 + (tid + it * NT) / (BN / 8), M - 1)];
    // copy rows read their own mask row: resolve the mask row pointers now, so the
    // epilogue's mask word is one load (state_mask / copy_kind lookups hide behind the K loop)
    if (xa.copy_kind != nullptr) {
#pragma unroll
      for (int it = 0; it < XIT; ++it)
        xstate[it] = xa.copy_kind[xstate[it]] ? -1 - min(m0 + (tid + it * NT) / (BN / 8), M - 1)
                                              : xa.state_mask[xstate[it]];
    } else {
#pragma unroll
      for (int it = 0; it < XIT; ++it) xstate[it] = xa.state_mask[xstate[it]];
    }
  }
  f32x4 acc[FM][FN];
  float ss[FM];
#pragma unroll
  for (int i = 0; i < FM; ++i) {
    ss[i] = 0.f;
#pragma unroll
    for (int j = 0; j < FN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  }

  // ---- K loop, ST-stage pipeline: the DMAs of the next ST-1 tiles are in flight
  // while tile kt is multiplied.  The wait is a constant counted vmcnt (this
  // wave's newest NI·(ST-1) resp. NI·(ST-2) DMAs may stay outstanding): past the last tile the
  // issue slot re-loads tile KT-1 into the idle buffer (never read) so the count
  // stays exact.  Raw s_barrier: a __syncthreads() would drain the DMA queue.
  const int KT = K / BKT;
  if constexpr (PROBE >= 3) {  // no loads at all: deterministic (zero) LDS operands
    for (int i = tid * 8; i < ST * TILE; i += NT * 8) *reinterpret_cast<uint4*>(smem + i) = make_uint4(0, 0, 0, 0);
    __syncthreads();
  }
#pragma unroll
  for (int s0 = 0; s0 < (PROBE >= 3 ? 0 : ST - 1); ++s0) {
    const int kk = min(s0, KT - 1) * BKT;
    issue_tile<BM, NW, BKT>(A, lda, m0, M - 1, kk, smem + s0 * TILE, wave, lane);
    issue_tile<BN, NW, BKT>(W, K, n0, N - 1, kk, smem + s0 * TILE + BM * BKT, wave, lane);
  }
  int cur = 0;
  if constexpr (ST == 2) {
    for (int kt = 0; kt < KT; ++kt) {
      const int nb = cur ^ 1;  // buffer of tile kt + 1 == (kt - 1) % 2
      const int kk = min(kt + 1, KT - 1) * BKT;
      if constexpr (PROBE != 2) {
        issue_tile<BM, NW, BKT>(A, lda, m0, M - 1, kk, smem + nb * TILE, wave, lane);
        issue_tile<BN, NW, BKT>(W, K, n0, N - 1, kk, smem + nb * TILE + BM * BKT, wave, lane);
        asm volatile("s_waitcnt vmcnt(%0)" ::"n"(NI) : "memory");  // tile kt landed (this wave's part)
      }
      __builtin_amdgcn_s_barrier();  // ... and every wave's part
      if constexpr (PROBE != 1)
        mma_tile<FM, FN, NORM, BKT>(acc, ss, smem + cur * TILE, smem + cur * TILE + BM * BKT, wm0, wn0, lane);
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      __builtin_amdgcn_s_barrier();  // WAR: buffer `cur` is re-filled by the next issue
      cur ^= 1;
    }
  } else {
    // >= 3 stages: ONE barrier per K-step.  Tile kt+ST-1 is issued after the barrier
    // into the buffer of tile kt-1, which every wave has finished reading by then.
    for (int kt = 0; kt < KT; ++kt) {
      asm volatile("s_waitcnt vmcnt(%0)" ::"n"(NI * (ST - 2)) : "memory");  // tile kt landed (this wave)
      __builtin_amdgcn_s_barrier();                                          // ... every wave; kt-1 read
      const int nb = cur == 0 ? ST - 1 : cur - 1;  // buffer of tile kt + ST - 1 == (kt - 1) % ST
      const int kk = min(kt + ST - 1, KT - 1) * BKT;
      issue_tile<BM, NW, BKT>(A, lda, m0, M - 1, kk, smem + nb * TILE, wave, lane);
      issue_tile<BN, NW, BKT>(W, K, n0, N - 1, kk, smem + nb * TILE + BM * BKT, wave, lane);
      mma_tile<FM, FN, NORM, BKT>(acc, ss, smem + cur * TILE, smem + cur * TILE + BM * BKT, wm0, wn0, lane);
      cur = cur + 1 == ST ? 0 : cur + 1;
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // the tail re-loads ...
  __syncthreads();  // ... of EVERY wave have landed before the C tile reuses the buffers
  if constexpr (EPI == 1 && !RPRE_EARLY) {
    load_rpre();
    asm volatile("" ::: "memory");  // issued here, not sunk to their first use
  }
  if constexpr (PROBE == 4) {
    float keep = 0.f;  // every accumulator stays live (no dead MFMAs)
#pragma unroll
    for (int i = 0; i < FM; ++i)
#pragma unroll
      for (int j = 0; j < FN; ++j) keep += acc[i][j][0] + acc[i][j][1] + acc[i][j][2] + acc[i][j][3] + ss[i];
    if (keep == 12345.f) C[tid] = 1;
    return;
  }

  // ---- row scales (RMSNorm): lanes l, l^16, l^32, l^48 hold the 4 k-quarters of
  // row l&15 — which is also the output row this lane holds (C^T layout), so the
  // scale never leaves registers
  float rsv[FM];
#pragma unroll
  for (int i = 0; i < FM; ++i) {
    rsv[i] = 1.f;
    if constexpr (NORM == 1) {
      float v = ss[i];
      v += __shfl_xor(v, 16, 64);
      v += __shfl_xor(v, 32, 64);
      rsv[i] = rsqrtf(v / (float)K + eps);
    } else if constexpr (NORM == 2) {
      float v = (ssv[i][0] + ssv[i][1]) + (ssv[i][2] + ssv[i][3]);
      v += __shfl_xor(v, 16, 64);
      v += __shfl_xor(v, 32, 64);
      rsv[i] = rsqrtf(v / (float)K + eps);
    }
  }

  // ---- epilogue 1: fragments -> bf16 tile in LDS (the K-loop buffers are free now).
  // Lane holds rows m = wm0 + 16i + (lane & 15), columns n0' + 4·(lane>>4) + r.
  uint16_t* Cs = smem;
  const int m_lane = lane & 15;
  const int c4 = (lane >> 4) * 4;
#pragma unroll
  for (int i = 0; i < FM; ++i) {
    const int row = wm0 + i * 16 + m_lane;
    const float sc = rsv[i];
    if constexpr (EPI == 2) {
#pragma unroll
      for (int j = 0; j < FN; j += 2) {
        const int col = (wn0 >> 1) + (j >> 1) * 16 + c4;
        float h[4];
#pragma unroll
        for (int r = 0; r < 4; ++r) h[r] = silu(acc[i][j][r] * sc) * (acc[i][j + 1][r] * sc);
        *reinterpret_cast<uint2*>(Cs + row * CST + col) =
            make_uint2((uint32_t)f2bf(h[0]) | ((uint32_t)f2bf(h[1]) << 16),
                       (uint32_t)f2bf(h[2]) | ((uint32_t)f2bf(h[3]) << 16));
      }
    } else {
#pragma unroll
      for (int j = 0; j < FN; ++j) {
        const int col = wn0 + j * 16 + c4;
        *reinterpret_cast<uint2*>(Cs + row * CST + col) =
            make_uint2((uint32_t)f2bf(acc[i][j][0] * sc) | ((uint32_t)f2bf(acc[i][j][1] * sc) << 16),
                       (uint32_t)f2bf(acc[i][j][2] * sc) | ((uint32_t)f2bf(acc[i][j][3] * sc) << 16));
      }
    }
  }
  __syncthreads();

  // ---- epilogue 2 (EPI 3): RoPE the q/k heads of this tile into q_out / the K
  // cache, or scatter the v heads into the blocked V^T cache.  Same rounding as
  // the unfused path: bf16 projection (the staged tile) -> fp32 RoPE -> bf16.
  if constexpr (EPI == 3) {
    const int h0 = (n0 >> 6) + ra.hb;
    if (h0 < ra.nh + ra.nkv) {
      // one (row, quarter) item per thread and trip: its (cos, sin) chunk is loaded once
      // and rotates that quarter of all HT heads of the tile (the heads share the row's
      // position)
#pragma unroll
      for (int it = 0; it < QIT; ++it) {
        const int q = tid + it * NT;
        if (q >= BM * 4) break;
        const int row = q >> 2, c = q & 3;
        const int gr = m0 + row;
        if (gr >= M) continue;
        const int p = epos[it];
        const float4* csp = reinterpret_cast<const float4*>(ra.cs + (size_t)(ra.p0 + p) * 32 + c * 8);
        float4 t[4];
#pragma unroll
        for (int e = 0; e < 4; ++e) t[e] = csp[e];  // (cos, sin) of dims 2e, 2e+1 of this chunk
#pragma unroll
        for (int j = 0; j < HT; ++j) {
          const int h = h0 + j;
          const uint4 v1 = *reinterpret_cast<const uint4*>(Cs + row * CST + j * 64 + c * 8);
          const uint4 v2 = *reinterpret_cast<const uint4*>(Cs + row * CST + j * 64 + 32 + c * 8);
          const uint32_t a1[4] = {v1.x, v1.y, v1.z, v1.w}, a2[4] = {v2.x, v2.y, v2.z, v2.w};
          uint32_t o1[4], o2[4];
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            const float x1l = bf2f(a1[e] & 0xffffu), x1h = bf2f(a1[e] >> 16);
            const float x2l = bf2f(a2[e] & 0xffffu), x2h = bf2f(a2[e] >> 16);
            o1[e] = (uint32_t)f2bf(x1l * t[e].x - x2l * t[e].y) | ((uint32_t)f2bf(x1h * t[e].z - x2h * t[e].w) << 16);
            o2[e] = (uint32_t)f2bf(x2l * t[e].x + x1l * t[e].y) | ((uint32_t)f2bf(x2h * t[e].z + x1h * t[e].w) << 16);
          }
          uint16_t* dst;
          if (h < ra.nh) dst = ra.q_out + ((size_t)gr * ra.nh + h) * 64;
          else dst = ra.k_cache + (((size_t)eslot[it] * ra.nkv + (h - ra.nh)) * ra.Lmax + p) * 64;
          *reinterpret_cast<uint4*>(dst + c * 8) = make_uint4(o1[0], o1[1], o1[2], o1[3]);
          *reinterpret_cast<uint4*>(dst + 32 + c * 8) = make_uint4(o2[0], o2[1], o2[2], o2[3]);
        }
      }
    } else {
      // one token per wave-instruction (lane = d).  The tile's positions / slots sit one
      // row per lane (prefetched before the K loop; a dependent scalar load per row
      // serialised ~16 L2 round trips per wave) and are broadcast with readlane: the
      // V^T address is a scalar base + 16 B x lane
      static_assert(BM <= 128, "V^T scatter: rows per lane register");
      const int kh0 = h0 - ra.nh - ra.nkv, nb = ra.Lmax >> 3;
      // (position, slot) of tile row r (wave-uniform r): broadcast from the lane registers
      auto pos_of = [&](int r) {
        return __builtin_amdgcn_readlane((BM > 64 && (r >> 6)) ? epos[VU - 1] : epos[0], r & 63);
      };
      auto slot_of = [&](int r) {
        return __builtin_amdgcn_readlane((BM > 64 && (r >> 6)) ? eslot[VU - 1] : eslot[0], r & 63);
      };
      for (int row = __builtin_amdgcn_readfirstlane(wave); row < BM; row += NW) {
        const int gr = m0 + row;
        if (gr >= M) break;
        const int p = pos_of(row), sl = slot_of(row);
        // V^T blocks hold 8 consecutive positions per dim: when the tile has all 8 rows of
        // this row's block (one sequence, positions 8k .. 8k+7), its first row writes them
        // as one 16-B chunk per dim and the others skip; partial blocks (sequence / tile
        // edges) are written element by element
        const int g = row - (p & 7);
        const bool full = g >= 0 && g + 7 < BM && m0 + g + 7 < M && slot_of(g) == sl && pos_of(g) == p - (p & 7) &&
                          slot_of(g + 7) == sl && pos_of(g + 7) == p - (p & 7) + 7;
        if (full && g != row) continue;
#pragma unroll
        for (int j = 0; j < HT; ++j) {
          const size_t base = (((size_t)sl * ra.nkv + kh0 + j) * nb + (p >> 3)) * 512;
          if (full) {
            uint32_t w[4];
#pragma unroll
            for (int e = 0; e < 4; ++e)
              w[e] = (uint32_t)Cs[(row + 2 * e) * CST + j * 64 + lane] |
                     ((uint32_t)Cs[(row + 2 * e + 1) * CST + j * 64 + lane] << 16);
            *reinterpret_cast<uint4*>(ra.vt_cache + base + (size_t)lane * 8) = make_uint4(w[0], w[1], w[2], w[3]);
          } else {
            ra.vt_cache[base + (p & 7) + (size_t)lane * 8] = Cs[row * CST + j * 64 + lane];
          }
        }
      }
    }
    return;
  }

  // ---- epilogue 2 (EPI 4): per-row masked arg-max of this tile's bf16 logits.
  // CPR lanes (consecutive, inside one wave) own one row's 8-column chunks.
  if constexpr (EPI == 4) {
    constexpr int CPR4 = BN / 8;
    static_assert(CPR4 <= 64 && (CPR4 & (CPR4 - 1)) == 0, "row chunks must fit a wave");
    static_assert((BM * CPR4) % NT == 0, "uniform epilogue trips");
    const int words = N >> 5;
#pragma unroll
    for (int it = 0; it < XIT; ++it) {
      const int q = tid + it * NT;
      const int row = q / CPR4, c = q % CPR4;
      const int gr = m0 + row;
      unsigned long long key = 0ull;
      if (gr < M) {
        const int col = n0 + c * 8;
        // xstate: the mask row of the state (>= 0) or -1 - row for a copy row
        const uint32_t* mrow = xstate[it] >= 0 ? xa.masks + (size_t)xstate[it] * words
                                               : xa.row_masks + (size_t)(-1 - xstate[it]) * words;
        const uint32_t bits = (mrow[col >> 5] >> (col & 31)) & 0xffu;
        if (bits) {
          const uint4 v = *reinterpret_cast<const uint4*>(Cs + row * CST + c * 8);
          const uint32_t w[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
          for (int e = 0; e < 8; ++e)
            if (bits & (1u << e)) {
              const unsigned long long k2 = argmax_key(bf2f((w[e >> 1] >> ((e & 1) * 16)) & 0xffffu), col + e);
              key = k2 > key ? k2 : key;
            }
        }
      }
#pragma unroll
      for (int o = CPR4 / 2; o > 0; o >>= 1) {
        const unsigned long long ok = __shfl_xor(key, o, 64);
        key = ok > key ? ok : key;
      }
      if (c == 0 && gr < M && key) atomicMax(xa.best + gr, key);
    }
    return;
  }

  // ---- epilogue 2: coalesced 16-B row chunks (+ residual)
  constexpr int CPR = BNO / 8;  // chunks per row
  const int c0 = EPI == 2 ? n0 / 2 : n0;
  if constexpr (EPI == 1) {
    // the CPR chunks of a row are CPR consecutive lanes of one wave, and every lane
    // runs the same trip count, so the row's x² partial reduces with shuffles (a
    // power-of-two CPR) or, for 96/192-wide tiles (CPR 12 / 24: a row's lanes are not
    // an aligned group), through a [BM][CPR] LDS image summed in a fixed order
    constexpr bool POW2 = (CPR & (CPR - 1)) == 0;
    // the shuffle reduction needs every lane on the same trip count
    static_assert(CPR <= 64 && (!POW2 || (BM * CPR) % NT == 0), "uniform epilogue trips");
    static_assert(POW2 || BM * CST + 2 * BM * CPR <= SMEM, "x² image fits beside the C tile");
    float* ssl = reinterpret_cast<float*>(smem + BM * CST);
    const bool want_ss = na.ssout != nullptr;
#pragma unroll
    for (int it = 0; it < RIT; ++it) {
      const int q = tid + it * NT;
      if (!POW2 && q >= BM * CPR) break;  // (the LDS path has no shuffles: ragged trips are fine)
      const int row = q / CPR, c = q % CPR;
      const int gr = m0 + row;
      float sq = 0.f;
      if (gr < M) {
        const uint4 v = *reinterpret_cast<const uint4*>(Cs + row * CST + c * 8);
        const uint4 rr = rpre[it];
        uint32_t a[4] = {v.x, v.y, v.z, v.w};
        const uint32_t b[4] = {rr.x, rr.y, rr.z, rr.w};
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const float lo = bf2f(a[e] & 0xffffu) + bf2f(b[e] & 0xffffu);
          const float hi = bf2f(a[e] >> 16) + bf2f(b[e] >> 16);
          a[e] = (uint32_t)f2bf(lo) | ((uint32_t)f2bf(hi) << 16);
          const float rl = bf2f(a[e] & 0xffffu), rh = bf2f(a[e] >> 16);  // the stored (rounded) values
          sq = fmaf(rl, rl, fmaf(rh, rh, sq));
        }
        *reinterpret_cast<uint4*>(C + (size_t)gr * ldc + c0 + c * 8) = make_uint4(a[0], a[1], a[2], a[3]);
      }
      if (want_ss) {
        if constexpr (POW2) {
#pragma unroll
          for (int o = 1; o < CPR; o <<= 1) sq += __shfl_xor(sq, o, 64);
          if (c == 0 && gr < M) na.ssout[(size_t)(n0 / BN) * na.ld + gr] = sq;
        } else {
          ssl[row * CPR + c] = sq;
        }
      }
    }
    if constexpr (!POW2) {
      // x² parts are 96 columns wide whatever the tile width: a 192-wide tile writes two
      // parts, each summed over its 12 chunks in the order a 96-wide tile sums them, so the
      // consumer's partials (and every row's result) do not depend on the tile config
      constexpr int PW = BN % 96 == 0 ? 96 : BN, CPP = PW / 8, NPART = BN / PW;
      if (want_ss) {
        __syncthreads();
        for (int q = tid; q < BM * NPART; q += NT) {
          const int r = q % BM, part = q / BM;
          if (m0 + r >= M) continue;
          float v = 0.f;
#pragma unroll
          for (int c = 0; c < CPP; ++c) v += ssl[r * CPR + part * CPP + c];
          na.ssout[(size_t)(n0 / PW + part) * na.ld + m0 + r] = v;
        }
      }
    }
    return;
  }
  for (int q = tid; q < BM * CPR; q += NT) {
    const int row = q / CPR, c = q % CPR;
    const int gr = m0 + row;
    if (gr >= M) continue;
    const uint4 v = *reinterpret_cast<const uint4*>(Cs + row * CST + c * 8);
    *reinterpret_cast<uint4*>(C + (size_t)gr * ldc + c0 + c * 8) = v;
  }
}

// ---------------------------------------------------------------------------
// 256x256 SwiGLU GEMM, 8 waves in two STAGGERED groups (cdna_hip_programming.md §5
// "256² 8-phase template", T3/T4/T5).  The 128²/2-barrier loop above tops out near
// 0.85 PFLOP/s: all waves read LDS together, then all multiply together.  Here
//
//  * wave (wr, wc) owns rows wr·128 + [0,128) and the two 32-column gate|up pairs
//    wc·32 + [0,32) ("lo", in W rows [0,128) of the tile) and 128 + wc·32 + [0,32)
//    ("hi"), so every wave needs the lo B half first and the hi half one phase later;
//  * a K-tile (BK 64) is four phases, one 64x32 quadrant (16 MFMAs) each:
//      p1 rows 0-63 x lo   (reads A0 + Blo)      p2 rows 64-127 x lo (reads A1)
//      p3 rows 64-127 x hi (reads Bhi)           p4 rows 0-63 x hi   (no LDS reads)
//    and each phase stages ONE 16 KB half-tile of the next K-tile (A_top, A_bot,
//    Blo, Bhi in p1..p4; 2 LDS-DMAs per wave) into the other of two 64 KB buffers;
//  * group wr = 1 runs one barrier behind group 0, so on every SIMD one wave's
//    MFMA cluster overlaps the other wave's LDS reads and DMA issue;
//  * RAW: a counted vmcnt(2) at the end of p4's read section retires A_top, A_bot
//    and Blo of the next tile (Bhi stays in flight), a vmcnt(4) at the end of p2
//    retires Bhi before p3 reads it; every such wait precedes, in both groups, the
//    barrier that precedes the first read.  WAR: a half-tile of tile t+1 is staged
//    only after every wave's last read of the same half of tile t-1 (A: p2, Blo: p1,
//    Bhi: p3; p4 reads nothing), which the lagging group completes two barriers
//    before the leading group's DMA.
// SwiGLU epilogue (EPI 2) with the row scale of NORM 0/1/2, as gemm_fused_kernel.
template <int NORM>
__global__ void __launch_bounds__(512) gemm256_swiglu_kernel(const uint16_t* __restrict__ A, int lda,
                                                            const uint16_t* __restrict__ W, uint16_t* C, int ldc,
                                                            int M, int N, int K, float eps, int tiles_m, int tiles_n,
                                                            int gm, NormArgs na) {
  constexpr int BM = 256, BN = 256, HALF = 128 * BK;  // elements per half-tile
  constexpr int BUF = 4 * HALF;                        // A_top, A_bot, Blo, Bhi
  constexpr int BNO = BN / 2, CST = BNO + 8;
  static_assert(BM * CST <= 2 * BUF, "C staging fits");
  // + the tile's 256 row sums of x² (NORM 2), one fp32 each, past the staging buffers
  // (ONE __shared__ array: cdna_hip_programming.md §5 trap 4a)
  __shared__ __attribute__((aligned(16))) uint16_t smem[2 * BUF + (NORM == 2 ? 2 * BM : 0)];
  float* ssl = reinterpret_cast<float*>(smem + 2 * BUF);

  const int T = tiles_m * tiles_n;
  const int orig = blockIdx.x, xcd = orig & 7, q8 = T >> 3, r8 = T & 7;
  const int t = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + (orig >> 3);
  const int gsz = gm * tiles_n, g = t / gsz, gl = t - g * gsz;
  const int grows = min(gm, tiles_m - g * gm);
  const int m0 = (g * gm + gl % grows) * BM;
  const int n0 = (gl / grows) * BN;

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wr = wave >> 2, wc = wave & 3;

  f32x4 acc[8][4];  // [16-row frag i][col frag j]: j 0,1 = lo pair (gate, up), 2,3 = hi pair
  float ss[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    ss[i] = 0.f;
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  }

  const int KT = K / BK;
  // half-tile h of K-tile kt into buffer b: A halves = A rows, B halves = W rows
  auto stage = [&](int b, int h, int kt) {
    const int kk = min(kt, KT - 1) * BK;  // past the end: re-load the last tile (idle buffer, never read)
    uint16_t* dst = smem + b * BUF + h * HALF;
    if (h < 2) issue_tile<128, 8>(A, lda, m0 + h * 128, M - 1, kk, dst, wave, lane);
    else issue_tile<128, 8>(W, K, n0 + (h - 2) * 128, N - 1, kk, dst, wave, lane);
  };
  // fragment reads: A frags of rows wr·128 + r0 + 16i, B frags of W rows wc·32 + 16j of half hb
  bf16x8 a0[2][4], a1[2][4], bq[2][2];
  auto read_a = [&](bf16x8 (&dst)[2][4], const uint16_t* base, int r0) {
#pragma unroll
    for (int s2 = 0; s2 < 2; ++s2)
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int row = r0 + i * 16 + (lane & 15), ch = s2 * 4 + (lane >> 4);
        dst[s2][i] = *reinterpret_cast<const bf16x8*>(base + row * BK + ((ch ^ (row & 7)) << 3));
      }
  };
  auto read_b = [&](const uint16_t* base) {
#pragma unroll
    for (int s2 = 0; s2 < 2; ++s2)
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        const int row = wc * 32 + j * 16 + (lane & 15), ch = s2 * 4 + (lane >> 4);
        bq[s2][j] = *reinterpret_cast<const bf16x8*>(base + row * BK + ((ch ^ (row & 7)) << 3));
      }
  };
  auto mfma_q = [&](bf16x8 (&af)[2][4], int i0, int j0) {
    __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int s2 = 0; s2 < 2; ++s2)
#pragma unroll
      for (int i = 0; i < 4; ++i) {
#pragma unroll
        for (int j = 0; j < 2; ++j)
          acc[i0 + i][j0 + j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bq[s2][j], af[s2][i], acc[i0 + i][j0 + j],
                                                                        0, 0, 0);
        if constexpr (NORM == 1)
          if (j0 == 0) ss[i0 + i] = sumsq_frag(af[s2][i], ss[i0 + i]);
      }
    __builtin_amdgcn_s_setprio(0);
  };
  auto mid = [&]() {  // end of a read section: barrier, then this wave's reads have landed
    __builtin_amdgcn_s_barrier();
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  };

  // prologue: K-tile 0 into buffer 0 (+ NORM 2: the rows' x² partials, summed into
  // LDS while the DMAs land — one thread per row, part-major loads are coalesced),
  // then group 1 falls one barrier behind
#pragma unroll
  for (int h = 0; h < 4; ++h) stage(0, h, 0);
  if constexpr (NORM == 2) {
    if (tid < BM) {
      const float* sp = na.ssin + min(m0 + tid, M - 1);
      float v[SS_PARTS];
#pragma unroll
      for (int p = 0; p < SS_PARTS; ++p) v[p] = sp[(size_t)p * na.ld];
      float tot = 0.f;
#pragma unroll
      for (int p = 0; p < SS_PARTS; ++p) tot += v[p];
      ssl[tid] = tot;
    }
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (__builtin_amdgcn_readfirstlane(wr) == 1) __builtin_amdgcn_s_barrier();

  for (int kt = 0; kt < KT; ++kt) {
    const int cb = kt & 1, nb = cb ^ 1;
    const uint16_t* buf = smem + cb * BUF;
    const uint16_t* abase = buf + wr * HALF;
    // p1: rows 0-63 x lo
    read_a(a0, abase, 0);
    read_b(buf + 2 * HALF);
    stage(nb, 0, kt + 1);
    mid();
    mfma_q(a0, 0, 0);
    __builtin_amdgcn_s_barrier();
    // p2: rows 64-127 x lo
    read_a(a1, abase, 64);
    stage(nb, 1, kt + 1);
    asm volatile("s_waitcnt vmcnt(4)" ::: "memory");  // Bhi of THIS tile (staged in the previous p4) landed
    mid();
    mfma_q(a1, 4, 0);
    __builtin_amdgcn_s_barrier();
    // p3: rows 64-127 x hi
    read_b(buf + 3 * HALF);
    stage(nb, 2, kt + 1);
    mid();
    mfma_q(a1, 4, 2);
    __builtin_amdgcn_s_barrier();
    // p4: rows 0-63 x hi (A0 still in registers: no LDS reads)
    stage(nb, 3, kt + 1);
    asm volatile("s_waitcnt vmcnt(2)" ::: "memory");  // A_top, A_bot, Blo of the next tile landed
    mid();
    mfma_q(a0, 0, 2);
    __builtin_amdgcn_s_barrier();
  }
  if (__builtin_amdgcn_readfirstlane(wr) == 0) __builtin_amdgcn_s_barrier();  // re-align the groups
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();

  // row scales: lane holds rows wr·128 + 16i + (lane & 15)
  float rsv[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    rsv[i] = 1.f;
    if constexpr (NORM == 1) {
      float v = ss[i];
      v += __shfl_xor(v, 16, 64);
      v += __shfl_xor(v, 32, 64);
      rsv[i] = rsqrtf(v / (float)K + eps);
    } else if constexpr (NORM == 2) {
      rsv[i] = rsqrtf(ssl[wr * 128 + i * 16 + (lane & 15)] / (float)K + eps);
    }
  }
  // SwiGLU into the staged bf16 tile: pair p (lo/hi) -> output cols p·64 + wc·16 + c4
  uint16_t* Cs = smem;
  const int c4 = (lane >> 4) * 4;
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    const int row = wr * 128 + i * 16 + (lane & 15);
#pragma unroll
    for (int p = 0; p < 2; ++p) {
      const int col = p * 64 + wc * 16 + c4;
      float h[4];
#pragma unroll
      for (int r = 0; r < 4; ++r) h[r] = silu(acc[i][2 * p][r] * rsv[i]) * (acc[i][2 * p + 1][r] * rsv[i]);
      *reinterpret_cast<uint2*>(Cs + row * CST + col) =
          make_uint2((uint32_t)f2bf(h[0]) | ((uint32_t)f2bf(h[1]) << 16),
                     (uint32_t)f2bf(h[2]) | ((uint32_t)f2bf(h[3]) << 16));
    }
  }
  __syncthreads();
  constexpr int CPR = BNO / 8;
  const int c0 = n0 / 2;
  for (int q = tid; q < BM * CPR; q += 512) {
    const int row = q / CPR, c = q % CPR;
    const int gr = m0 + row;
    if (gr >= M) continue;
    *reinterpret_cast<uint4*>(C + (size_t)gr * ldc + c0 + c * 8) =
        *reinterpret_cast<const uint4*>(Cs + row * CST + c * 8);
  }
}

// Persistent form of gemm256_swiglu_kernel (cfg 20): one block per CU walks its tiles
// (virtual ids blockIdx.x + k·gridDim.x through the same XCD-aware map), and the
// per-tile fixed cost — first K-tile load, SwiGLU epilogue, output stores — is
// overlapped with the neighbouring tiles' K loops: the last K-tile of tile i stages
// K-tile 0 of tile i+1 (and, NORM 2, its rows' x² partials: 16 × 1 KB LDS-DMAs into
// `raw`, summed into `ssl` by group 0 after the loop), the epilogue stores straight
// from the accumulators (no LDS staging, so nothing waits for the stores), and the
// wave groups stay staggered across tiles.  Same phase / wait structure as above
// except (a) p4 re-reads A rows 0-63 (one A register set: the kernel then fits 256
// VGPRs without spills) and (b) the last K-tile's p2 wait, vmcnt(6): the 2 partial
// DMAs of p1 precede A_top.
//
// TWOA (cfg 42, A/B): both A register sets kept (rows 0-63 from p1 through p4, rows
// 64-127 in p2 / p3), so p4 issues no LDS reads -- 32 VGPRs more per lane.
template <int NORM, bool TWOA = false>
__global__ void __launch_bounds__(512) gemm256p_swiglu_kernel(const uint16_t* __restrict__ A, int lda,
                                                             const uint16_t* __restrict__ W, uint16_t* C, int ldc,
                                                             int M, int N, int K, float eps, int tiles_m, int tiles_n,
                                                             int gm, NormArgs na) {
  constexpr int BM = 256, BN = 256, HALF = 128 * BK, BUF = 4 * HALF;
  constexpr int RAW = NORM == 2 ? SS_PARTS * BM * 2 : 0;  // [16][256] fp32, in uint16 units
  constexpr int SSL = NORM == 2 ? 2 * BM * 2 : 0;         // [2][256] fp32 (tile parity)
  __shared__ __attribute__((aligned(16))) uint16_t smem[2 * BUF + RAW + SSL];
  float* raw = reinterpret_cast<float*>(smem + 2 * BUF);
  float* ssl = reinterpret_cast<float*>(smem + 2 * BUF + RAW);

  const int T = tiles_m * tiles_n;
  auto tile_mn = [&](int v, int& m0, int& n0) {
    const int xcd = v & 7, q8 = T >> 3, r8 = T & 7;
    const int t = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + (v >> 3);
    const int gsz = gm * tiles_n, g = t / gsz, gl = t - g * gsz;
    const int grows = min(gm, tiles_m - g * gm);
    m0 = (g * gm + gl % grows) * BM;
    n0 = (gl / grows) * BN;
  };
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wr = wave >> 2, wc = wave & 3;
  const int KT = K / BK;

  auto stage = [&](int b, int h, int mm, int nn, int kt) {
    const int kk = min(kt, KT - 1) * BK;
    uint16_t* dst = smem + b * BUF + h * HALF;
    if (h < 2) issue_tile<128, 8>(A, lda, mm + h * 128, M - 1, kk, dst, wave, lane);
    else issue_tile<128, 8>(W, K, nn + (h - 2) * 128, N - 1, kk, dst, wave, lane);
  };
  // NORM 2: parts 2w, 2w+1 of rows mm + [0, 256): lane l -> rows mm + 4l .. +3 (16 B);
  // groups past the end re-read the last aligned group (never used); ld % 4 == 0
  auto stage_ss = [&](int mm) {
    if constexpr (NORM == 2) {
      const int r = min(mm + lane * 4, ((M + 3) & ~3) - 4);
#pragma unroll
      for (int e = 0; e < 2; ++e) {
        const int p = wave * 2 + e;
        __builtin_amdgcn_global_load_lds((const void*)(na.ssin + (size_t)p * na.ld + r),
                                         (lds_ptr_t)(raw + p * BM), 16, 0, 0);
      }
    }
  };
  auto sum_ss = [&](int par) {  // group 0: one row per thread
    if constexpr (NORM == 2) {
      if (tid < BM) {
        float v = 0.f;
#pragma unroll
        for (int p = 0; p < SS_PARTS; ++p) v += raw[p * BM + tid];
        ssl[par * BM + tid] = v;
      }
    }
  };

  f32x4 acc[8][4];
  float ss[8];
  auto zero_acc = [&]() {
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      ss[i] = 0.f;
#pragma unroll
      for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
    }
  };
  bf16x8 af[2][4], bq[2][2];  // ONE A set (p4 re-reads rows 0-63): 32 VGPRs fewer, no spills
  bf16x8 ab[2][4];             // TWOA: rows 64-127 (unused otherwise)
  auto read_a = [&](bf16x8 (&dst)[2][4], const uint16_t* base, int r0) {
#pragma unroll
    for (int s2 = 0; s2 < 2; ++s2)
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int row = r0 + i * 16 + (lane & 15), ch = s2 * 4 + (lane >> 4);
        dst[s2][i] = *reinterpret_cast<const bf16x8*>(base + row * BK + ((ch ^ (row & 7)) << 3));
      }
  };
  auto read_b = [&](const uint16_t* base) {
#pragma unroll
    for (int s2 = 0; s2 < 2; ++s2)
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        const int row = wc * 32 + j * 16 + (lane & 15), ch = s2 * 4 + (lane >> 4);
        bq[s2][j] = *reinterpret_cast<const bf16x8*>(base + row * BK + ((ch ^ (row & 7)) << 3));
      }
  };
  auto mfma_q = [&](bf16x8 (&a_)[2][4], int i0, int j0) {
    __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int s2 = 0; s2 < 2; ++s2)
#pragma unroll
      for (int i = 0; i < 4; ++i) {
#pragma unroll
        for (int j = 0; j < 2; ++j)
          acc[i0 + i][j0 + j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bq[s2][j], a_[s2][i], acc[i0 + i][j0 + j],
                                                                        0, 0, 0);
        if constexpr (NORM == 1)
          if (j0 == 0) ss[i0 + i] = sumsq_frag(a_[s2][i], ss[i0 + i]);
      }
    __builtin_amdgcn_s_setprio(0);
  };
  auto mid = [&]() {
    __builtin_amdgcn_s_barrier();
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  };

  int v = blockIdx.x;
  if (v >= T) return;  // (the launcher sizes the grid <= T: never taken)
  int m0, n0;
  tile_mn(v, m0, n0);
#pragma unroll
  for (int h = 0; h < 4; ++h) stage(0, h, m0, n0, 0);
  stage_ss(m0);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  sum_ss(0);
  __syncthreads();
  zero_acc();
  if (__builtin_amdgcn_readfirstlane(wr) == 1) __builtin_amdgcn_s_barrier();

  int gk = 0, tpar = 0;
  const int c4 = (lane >> 4) * 4;
  while (true) {
    const int vn = v + gridDim.x;
    const bool more = vn < T;
    int m1 = m0, n1 = n0;
    if (more) tile_mn(vn, m1, n1);
    for (int kt = 0; kt < KT; ++kt, ++gk) {
      const int cb = gk & 1, nb = cb ^ 1;
      const bool last = kt == KT - 1;
      const int sm = last ? m1 : m0, sn = last ? n1 : n0, sk = last ? (more ? 0 : KT - 1) : kt + 1;
      const uint16_t* buf = smem + cb * BUF;
      const uint16_t* abase = buf + wr * HALF;
      // p1: rows 0-63 x lo
      read_a(af, abase, 0);
      read_b(buf + 2 * HALF);
      if (last) stage_ss(sm);
      stage(nb, 0, sm, sn, sk);
      mid();
      mfma_q(af, 0, 0);
      __builtin_amdgcn_s_barrier();
      // p2: rows 64-127 x lo
      if constexpr (TWOA) read_a(ab, abase, 64);
      else read_a(af, abase, 64);
      stage(nb, 1, sm, sn, sk);
      if (NORM == 2 && last) asm volatile("s_waitcnt vmcnt(6)" ::: "memory");  // + this p1's partial DMAs
      else asm volatile("s_waitcnt vmcnt(4)" ::: "memory");                    // Bhi of THIS K-tile landed
      mid();
      if constexpr (TWOA) mfma_q(ab, 4, 0);
      else mfma_q(af, 4, 0);
      __builtin_amdgcn_s_barrier();
      // p3: rows 64-127 x hi
      read_b(buf + 3 * HALF);
      stage(nb, 2, sm, sn, sk);
      mid();
      if constexpr (TWOA) mfma_q(ab, 4, 2);
      else mfma_q(af, 4, 2);
      __builtin_amdgcn_s_barrier();
      // p4: rows 0-63 x hi (re-read: WAR-safe, the next DMA into this A half is staged
      // after the lagging group's p4 barrier)
      if constexpr (!TWOA) read_a(af, abase, 0);
      stage(nb, 3, sm, sn, sk);
      asm volatile("s_waitcnt vmcnt(2)" ::: "memory");  // next K-tile's A_top, A_bot, Blo (+ partials)
      mid();
      mfma_q(af, 0, 2);
      __builtin_amdgcn_s_barrier();
    }
    // next tile's row sums (its partials landed: every wave's p4 wait precedes a barrier
    // this wave has passed); this tile's are in ssl[tpar]
    if (more) sum_ss(tpar ^ 1);
    // epilogue straight from the accumulators: row m0 + wr·128 + 16i + (lane & 15),
    // SwiGLU pair p -> output columns n0/2 + p·64 + wc·16 + c4 .. +3
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const int rl = wr * 128 + i * 16 + (lane & 15);
      float rs = 1.f;
      if constexpr (NORM == 1) {
        float x = ss[i];
        x += __shfl_xor(x, 16, 64);
        x += __shfl_xor(x, 32, 64);
        rs = rsqrtf(x / (float)K + eps);
      } else if constexpr (NORM == 2) {
        rs = rsqrtf(ssl[tpar * BM + rl] / (float)K + eps);
      }
      const int gr = m0 + rl;
      if (gr < M) {
#pragma unroll
        for (int p = 0; p < 2; ++p) {
          float h[4];
#pragma unroll
          for (int r = 0; r < 4; ++r) h[r] = silu(acc[i][2 * p][r] * rs) * (acc[i][2 * p + 1][r] * rs);
          *reinterpret_cast<uint2*>(C + (size_t)gr * ldc + n0 / 2 + p * 64 + wc * 16 + c4) =
              make_uint2((uint32_t)f2bf(h[0]) | ((uint32_t)f2bf(h[1]) << 16),
                         (uint32_t)f2bf(h[2]) | ((uint32_t)f2bf(h[3]) << 16));
        }
      }
    }
    if (!more) break;
    zero_acc();
    v = vn;
    m0 = m1;
    n0 = n1;
    tpar ^= 1;
  }
  if (__builtin_amdgcn_readfirstlane(wr) == 0) __builtin_amdgcn_s_barrier();  // re-align the groups
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // the dummy tail DMAs
}

// Persistent QK+RoPE GEMM (cfg 39): the gate/up kernel's schedule (one block per CU,
// two staggered 4-wave groups, 4 phases per BK 64 K-tile, the next tile's first K-tile
// staged during this one's last) for the q and k heads of the QKV projection (N =
// (nh + nkv)·64, a multiple of 256: 4 heads per tile).  W rows are loaded in the RoPE-pair
// order (stage), so the epilogue rotates in registers and stores q rows / K-cache rows
// straight from the accumulators; the rows' positions and slots are LDS-DMA'd with the
// next tile's first K-tile (psl, tile parity).  The v heads go through cfg 28
// (sg_gemm_qkv_rope).
template <int NORM>
__global__ void __launch_bounds__(512) gemm256p_qk_rope_kernel(const uint16_t* __restrict__ A, int lda,
                                                              const uint16_t* __restrict__ W, int M, int N, int K,
                                                              float eps, int tiles_m, int tiles_n, int gm, NormArgs na,
                                                              RopeArgs ra) {
  constexpr int BM = 256, BN = 256, HALF = 128 * BK, BUF = 4 * HALF;
  constexpr int RAW = NORM == 2 ? SS_PARTS * BM * 2 : 0;  // [16][256] fp32, in uint16 units
  constexpr int SSL = NORM == 2 ? 2 * BM * 2 : 0;         // [2][256] fp32 (tile parity)
  constexpr int PSL = 2 * 2 * BM * 2;                      // [2 parity][pos, slot][256] int32
  __shared__ __attribute__((aligned(16))) uint16_t smem[2 * BUF + RAW + SSL + PSL];
  float* raw = reinterpret_cast<float*>(smem + 2 * BUF);
  float* ssl = reinterpret_cast<float*>(smem + 2 * BUF + RAW);
  int* psl = reinterpret_cast<int*>(smem + 2 * BUF + RAW + SSL);

  const int T = tiles_m * tiles_n;
  auto tile_mn = [&](int v, int& m0, int& n0) {
    const int xcd = v & 7, q8 = T >> 3, r8 = T & 7;
    const int t = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + (v >> 3);
    const int gsz = gm * tiles_n, g = t / gsz, gl = t - g * gsz;
    const int grows = min(gm, tiles_m - g * gm);
    m0 = (g * gm + gl % grows) * BM;
    n0 = (gl / grows) * BN;
  };
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wr = wave >> 2, wc = wave & 3;
  const int KT = K / BK;

  // W rows in the RoPE-pair order: tile row t of half hh holds head n0/64 + wc of dims
  // hh·16 + jj·32 + [0, 16) (wc = (t & 127) >> 5, jj = bit 4), so a wave's fragments j 0 / 1
  // (and 2 / 3) are the dims d and d + 32 of ONE head: the rotation stays in the lane
  auto stage = [&](int b, int h, int mm, int nn, int kt) {
    const int kk = min(kt, KT - 1) * BK;
    uint16_t* dst = smem + b * BUF + h * HALF;
    if (h < 2) {
      issue_tile<128, 8>(A, lda, mm + h * 128, M - 1, kk, dst, wave, lane);
    } else {
      const int hh = h - 2, rr = lane >> 3, pc = lane & 7;
#pragma unroll
      for (int i = 0; i < 2; ++i) {
        const int g = wave + 8 * i, row = 8 * g + rr;  // 8-row piece g of this half
        const int src = nn + (row >> 5) * 64 + hh * 16 + ((row >> 4) & 1) * 32 + (row & 15);
        const uint16_t* gp = W + (size_t)src * K + kk + ((pc ^ (row & 7)) << 3);
        __builtin_amdgcn_global_load_lds((const void*)gp, (lds_ptr_t)(dst + g * 8 * BK), 16, 0, 0);
      }
    }
  };
  // the rows' positions / KV slots of tile rows mm + [0, 256) into psl[par]: wave w loads
  // array w >> 2, rows (w & 3)·64 + lane -- one dword LDS-DMA per wave (rows past the end
  // re-read row M - 1, never used)
  auto stage_ps = [&](int mm, int par) {
    const int arr = wave >> 2, row = min(mm + (wave & 3) * 64 + lane, M - 1);
    const int* src = (arr ? ra.slot : ra.pos) + row;
    __builtin_amdgcn_global_load_lds((const void*)src, (lds_ptr_t)(psl + (par * 2 + arr) * BM + (wave & 3) * 64), 4, 0,
                                     0);
  };
  // NORM 2: parts 2w, 2w+1 of rows mm + [0, 256): lane l -> rows mm + 4l .. +3 (16 B);
  // groups past the end re-read the last aligned group (never used); ld % 4 == 0
  auto stage_ss = [&](int mm) {
    if constexpr (NORM == 2) {
      const int r = min(mm + lane * 4, ((M + 3) & ~3) - 4);
#pragma unroll
      for (int e = 0; e < 2; ++e) {
        const int p = wave * 2 + e;
        __builtin_amdgcn_global_load_lds((const void*)(na.ssin + (size_t)p * na.ld + r),
                                         (lds_ptr_t)(raw + p * BM), 16, 0, 0);
      }
    }
  };
  auto sum_ss = [&](int par) {  // group 0: one row per thread
    if constexpr (NORM == 2) {
      if (tid < BM) {
        float v = 0.f;
#pragma unroll
        for (int p = 0; p < SS_PARTS; ++p) v += raw[p * BM + tid];
        ssl[par * BM + tid] = v;
      }
    }
  };

  f32x4 acc[8][4];
  float ss[8];
  auto zero_acc = [&]() {
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      ss[i] = 0.f;
#pragma unroll
      for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
    }
  };
  bf16x8 af[2][4], bq[2][2];  // ONE A set (p4 re-reads rows 0-63): 32 VGPRs fewer, no spills
  auto read_a = [&](bf16x8 (&dst)[2][4], const uint16_t* base, int r0) {
#pragma unroll
    for (int s2 = 0; s2 < 2; ++s2)
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int row = r0 + i * 16 + (lane & 15), ch = s2 * 4 + (lane >> 4);
        dst[s2][i] = *reinterpret_cast<const bf16x8*>(base + row * BK + ((ch ^ (row & 7)) << 3));
      }
  };
  auto read_b = [&](const uint16_t* base) {
#pragma unroll
    for (int s2 = 0; s2 < 2; ++s2)
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        const int row = wc * 32 + j * 16 + (lane & 15), ch = s2 * 4 + (lane >> 4);
        bq[s2][j] = *reinterpret_cast<const bf16x8*>(base + row * BK + ((ch ^ (row & 7)) << 3));
      }
  };
  auto mfma_q = [&](bf16x8 (&a_)[2][4], int i0, int j0) {
    __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int s2 = 0; s2 < 2; ++s2)
#pragma unroll
      for (int i = 0; i < 4; ++i) {
#pragma unroll
        for (int j = 0; j < 2; ++j)
          acc[i0 + i][j0 + j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bq[s2][j], a_[s2][i], acc[i0 + i][j0 + j],
                                                                        0, 0, 0);
        if constexpr (NORM == 1)
          if (j0 == 0) ss[i0 + i] = sumsq_frag(a_[s2][i], ss[i0 + i]);
      }
    __builtin_amdgcn_s_setprio(0);
  };
  auto mid = [&]() {
    __builtin_amdgcn_s_barrier();
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  };

  int v = blockIdx.x;
  if (v >= T) return;  // (the launcher sizes the grid <= T: never taken)
  int m0, n0;
  tile_mn(v, m0, n0);
#pragma unroll
  for (int h = 0; h < 4; ++h) stage(0, h, m0, n0, 0);
  stage_ss(m0);
  stage_ps(m0, 0);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  sum_ss(0);
  __syncthreads();
  zero_acc();
  if (__builtin_amdgcn_readfirstlane(wr) == 1) __builtin_amdgcn_s_barrier();

  int gk = 0, tpar = 0;
  const int c4 = (lane >> 4) * 4;
  while (true) {
    const int vn = v + gridDim.x;
    const bool more = vn < T;
    int m1 = m0, n1 = n0;
    if (more) tile_mn(vn, m1, n1);
    for (int kt = 0; kt < KT; ++kt, ++gk) {
      const int cb = gk & 1, nb = cb ^ 1;
      const bool last = kt == KT - 1;
      const int sm = last ? m1 : m0, sn = last ? n1 : n0, sk = last ? (more ? 0 : KT - 1) : kt + 1;
      const uint16_t* buf = smem + cb * BUF;
      const uint16_t* abase = buf + wr * HALF;
      // p1: rows 0-63 x lo
      read_a(af, abase, 0);
      read_b(buf + 2 * HALF);
      if (last) {
        stage_ss(sm);
        stage_ps(sm, tpar ^ 1);
      }
      stage(nb, 0, sm, sn, sk);
      mid();
      mfma_q(af, 0, 0);
      __builtin_amdgcn_s_barrier();
      // p2: rows 64-127 x lo
      read_a(af, abase, 64);
      stage(nb, 1, sm, sn, sk);
      if (NORM == 2 && last) asm volatile("s_waitcnt vmcnt(7)" ::: "memory");  // + this p1's partial / pos DMAs
      else if (last) asm volatile("s_waitcnt vmcnt(5)" ::: "memory");          // + this p1's pos / slot DMA
      else asm volatile("s_waitcnt vmcnt(4)" ::: "memory");                    // Bhi of THIS K-tile landed
      mid();
      mfma_q(af, 4, 0);
      __builtin_amdgcn_s_barrier();
      // p3: rows 64-127 x hi
      read_b(buf + 3 * HALF);
      stage(nb, 2, sm, sn, sk);
      mid();
      mfma_q(af, 4, 2);
      __builtin_amdgcn_s_barrier();
      // p4: rows 0-63 x hi (re-read: WAR-safe, the next DMA into this A half is staged
      // after the lagging group's p4 barrier)
      read_a(af, abase, 0);
      stage(nb, 3, sm, sn, sk);
      asm volatile("s_waitcnt vmcnt(2)" ::: "memory");  // next K-tile's A_top, A_bot, Blo (+ partials)
      mid();
      mfma_q(af, 0, 2);
      __builtin_amdgcn_s_barrier();
    }
    // the tile's (cos, sin) table rows into the K-tile buffer the last K-step read (64 KB:
    // 256 rows x 32 float2) -- the epilogue then loads nothing from global memory, so its
    // stores never wait (a global load would wait for every older vector-memory op of the
    // wave, vmcnt retires in order: the next tile's prefetch and the previous stores).
    // Group 0 first passes one barrier (pairing group 1's last K-step barrier: both
    // groups' reads of that buffer are done), then each wave DMAs 32 rows, 16-B chunk c
    // of row r at slot c ^ (r & 15) (conflict-free reads below)
    if (__builtin_amdgcn_readfirstlane(wr) == 0) __builtin_amdgcn_s_barrier();
    const int* pp = psl + (tpar * 2) * BM;
    const int* sp = psl + (tpar * 2 + 1) * BM;
    uint16_t* cbuf = smem + ((gk - 1) & 1) * BUF;
#pragma unroll
    for (int d = 0; d < 8; ++d) {
      const int r = wave * 32 + d * 4 + (lane >> 4), c = (lane & 15) ^ (r & 15);
      const float2* src = ra.cs + (size_t)(ra.p0 + pp[r]) * 32 + c * 2;
      __builtin_amdgcn_global_load_lds((const void*)src, (lds_ptr_t)(cbuf + (wave * 32 + d * 4) * 128), 16, 0, 0);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();  // every wave's table rows landed (groups aligned from here)
    // next tile's row sums (its partials landed before the barrier above); this tile's
    // are in ssl[tpar]
    if (more) sum_ss(tpar ^ 1);
    // epilogue straight from the accumulators: row m0 + wr·128 + 16i + (lane & 15) of head
    // n0/64 + wc, dims dh + c4 .. +3 (x1) and their partners dh + 32 + c4 .. (x2), dh = 0
    // (fragments 0 / 1) and 16 (fragments 2 / 3).  The unfused path's rounding: bf16
    // projection, fp32 rotation, bf16
    const int h = (n0 >> 6) + wc;
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const int rl = wr * 128 + i * 16 + (lane & 15);
      float rs = 1.f;
      if constexpr (NORM == 1) {
        float x = ss[i];
        x += __shfl_xor(x, 16, 64);
        x += __shfl_xor(x, 32, 64);
        rs = rsqrtf(x / (float)K + eps);
      } else if constexpr (NORM == 2) {
        rs = rsqrtf(ssl[tpar * BM + rl] / (float)K + eps);
      }
      const int gr = m0 + rl;
      if (gr < M) {
        const int p = pp[rl];
        uint16_t* dst = h < ra.nh ? ra.q_out + ((size_t)gr * ra.nh + h) * 64
                                  : ra.k_cache + (((size_t)sp[rl] * ra.nkv + (h - ra.nh)) * ra.Lmax + p) * 64;
#pragma unroll
        for (int a = 0; a < 2; ++a) {  // dims a·16 + c4 .. +3 and their +32 partners
          const int c0 = a * 8 + (c4 >> 1);  // 16-B chunk of dims a·16 + c4, c4 + 1
          const float4 t0 = *reinterpret_cast<const float4*>(cbuf + rl * 128 + ((c0 ^ (rl & 15)) << 3));
          const float4 t1 = *reinterpret_cast<const float4*>(cbuf + rl * 128 + (((c0 + 1) ^ (rl & 15)) << 3));
          const float cs4[8] = {t0.x, t0.y, t0.z, t0.w, t1.x, t1.y, t1.z, t1.w};
          uint32_t o1[2], o2[2];
#pragma unroll
          for (int e = 0; e < 2; ++e) {
            float r1[2], r2[2];
#pragma unroll
            for (int u = 0; u < 2; ++u) {
              const int r = 2 * e + u;
              const float x1 = bf2f(f2bf(acc[i][2 * a][r] * rs)), x2 = bf2f(f2bf(acc[i][2 * a + 1][r] * rs));
              const float c = cs4[2 * r], sn = cs4[2 * r + 1];
              r1[u] = x1 * c - x2 * sn;
              r2[u] = x2 * c + x1 * sn;
            }
            o1[e] = (uint32_t)f2bf(r1[0]) | ((uint32_t)f2bf(r1[1]) << 16);
            o2[e] = (uint32_t)f2bf(r2[0]) | ((uint32_t)f2bf(r2[1]) << 16);
          }
          *reinterpret_cast<uint2*>(dst + a * 16 + c4) = make_uint2(o1[0], o1[1]);
          *reinterpret_cast<uint2*>(dst + 32 + a * 16 + c4) = make_uint2(o2[0], o2[1]);
        }
      }
    }
    if (!more) break;  // (the groups are aligned: no re-align barrier at the end)
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();  // every wave read its table rows: the next tile's DMAs may refill the buffer
    if (__builtin_amdgcn_readfirstlane(wr) == 1) __builtin_amdgcn_s_barrier();  // group 1 falls behind again
    zero_acc();
    v = vn;
    m0 = m1;
    n0 = n1;
    tpar ^= 1;
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // the dummy tail DMAs
}

// ---------------------------------------------------------------------------
// Persistent, STAGGERED 256x192 residual GEMM (cfg 35): C = R + A·Wᵀ for the N = 576
// residual GEMMs (o-proj, down-proj), the residual counterpart of the gate/up kernel's
// schedule (the one-group read-then-multiply loop of cfg 28 kept
// both at 24-29 % of the dense peak).
//
//  * 8 waves in two groups; group wr owns tile rows wr·128 + [0,128) and runs ONE
//    barrier behind the other, so on every SIMD one wave's MFMA cluster overlaps the
//    other wave's LDS reads (2 waves per SIMD);
//  * wave (wr, wi, wj) computes rows wr·128 + wi·64 + [0,64) x columns wj·96 + [0,96):
//    64x96 wave tiles (cfg 28's), 4 x 6 fragments of 16x16x32 MFMAs;
//  * BK 32 K-steps (64-B LDS rows, the sw32 swizzle) in NB ring buffers of 28 KB
//    (A 256 rows + W 192 rows); a step's 4 LDS-DMAs per wave are issued NB-1 steps
//    ahead, right AFTER the barrier that ends a read section (the lagging group's reads
//    of the buffer being refilled have retired: it waits lgkmcnt(0) before its next
//    barrier), and retired by a counted vmcnt one step before the step is read (every
//    wave's wait precedes a barrier that precedes any read of that step);
//  * persistent: one block per CU walks its tiles through the same XCD-aware grouped map,
//    the step sequence runs on across tiles (the next tile's first K-steps are in flight
//    during this tile's last), and the epilogue works from the accumulators: residual add
//    with the unfused path's rounding (bf16 product, fp32 add, bf16), 8-byte stores, and
//    the output rows' x² partials per 96-column part in the EXACT order of the 96-wide
//    tiles (pairs (2e, 2e+1) of an 8-column chunk by fmaf chains, chunks summed left to
//    right), so every consumer sees the same partials whichever tile produced them.
// MF 32: the same tile with v_mfma_f32_32x32x16_bf16 (2 x 3 fragments of 32x32 per wave;
// VERDICT r05 next #2's A/B): the same 10 fragment reads per K-step (the wave tile, not
// the MFMA shape, sets the LDS traffic) for 12 instead of 24 MFMAs.
template <int NB, int MF, bool STAG = true>
__global__ void __launch_bounds__(512) gemm256p_resid_kernel(const uint16_t* __restrict__ A, int lda,
                                                            const uint16_t* __restrict__ W, uint16_t* C, int ldc,
                                                            const uint16_t* R, int ldr, int M, int N, int K,
                                                            int tiles_m, int tiles_n, int gm, NormArgs na) {
  constexpr int BM = 256, BN = 192, BKT = 32, BUF = (BM + BN) * BKT;
  static_assert(NB >= 4 && NB * BUF * 2 <= 160 * 1024, "ring buffers");
  static_assert(MF == 16 || MF == 32, "MFMA shape");
  constexpr int FI = 64 / MF, FJ = 96 / MF;  // fragments per wave tile
  typedef float f32x16 __attribute__((ext_vector_type(16)));
  typedef typename std::conditional<MF == 16, f32x4, f32x16>::type accv;
  constexpr int AV = MF == 16 ? 4 : 16;  // accumulator values per lane per fragment
  constexpr int KS = MF == 16 ? 1 : 2;   // MFMA k-substeps per BK 32 step
  __shared__ __attribute__((aligned(16))) uint16_t smem[NB * BUF];

  const int T = tiles_m * tiles_n;
  auto tile_mn = [&](int v, int& m0, int& n0) {
    const int xcd = v & 7, q8 = T >> 3, r8 = T & 7;
    const int t = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + (v >> 3);
    const int gsz = gm * tiles_n, g = t / gsz, gl = t - g * gsz;
    const int grows = min(gm, tiles_m - g * gm);
    m0 = (g * gm + gl % grows) * BM;
    n0 = (gl / grows) * BN;
  };
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wr = wave >> 2, wi = (wave >> 1) & 1, wj = wave & 1;
  const int rbase = wr * 128 + wi * 64, cbase = wj * 96;
  const int KT = K / BKT;
  const int G = gridDim.x;
  if ((int)blockIdx.x >= T) return;  // (the launcher sizes the grid <= T: never taken)
  const int my_tiles = (T - (int)blockIdx.x + G - 1) / G;
  const int S = my_tiles * KT;  // K-steps of this block, over all its tiles

  // step t's DMAs (4 per wave) into buffer t % NB; steps past the end re-load the last
  // one (same bytes, an idle buffer, never read) so every wave's vmcnt stays exact
  auto stage = [&](int t) {
    const int tt = min(t, S - 1);
    int mm, nn;
    tile_mn((int)blockIdx.x + (tt / KT) * G, mm, nn);
    const int kk = (tt % KT) * BKT;
    uint16_t* dst = smem + (t % NB) * BUF;
    issue_tile<BM, 8, BKT>(A, lda, mm, M - 1, kk, dst, wave, lane);
    issue_tile<BN, 8, BKT>(W, K, nn, N - 1, kk, dst + BM * BKT, wave, lane);
  };
  accv acc[FI][FJ];
  auto zero_acc = [&]() {
#pragma unroll
    for (int i = 0; i < FI; ++i)
#pragma unroll
      for (int j = 0; j < FJ; ++j)
#pragma unroll
        for (int q = 0; q < AV; ++q) acc[i][j][q] = 0.f;
  };
  zero_acc();
  bf16x8 af[KS][FI], bq[KS][FJ];
  uint2 rres[FI][FJ * (AV / 4)];  // the tile's residual chunks (requested on its last K-step)
  // MF 16: lane reads 16-B chunk (lane >> 4) of row (lane & 15); MF 32: chunk
  // 2·ks + (lane >> 5) of row (lane & 31)
  auto read_frags = [&](const uint16_t* buf) {
#pragma unroll
    for (int ks = 0; ks < KS; ++ks) {
      const int ch = MF == 16 ? (lane >> 4) : 2 * ks + (lane >> 5);
      const int rl = lane & (MF - 1);
#pragma unroll
      for (int i = 0; i < FI; ++i) {
        const int row = rbase + i * MF + rl;
        af[ks][i] = *reinterpret_cast<const bf16x8*>(buf + row * BKT + ((ch ^ sw32(row)) << 3));
      }
      const uint16_t* bb = buf + BM * BKT;
#pragma unroll
      for (int j = 0; j < FJ; ++j) {
        const int row = cbase + j * MF + rl;
        bq[ks][j] = *reinterpret_cast<const bf16x8*>(bb + row * BKT + ((ch ^ sw32(row)) << 3));
      }
    }
  };

  // prologue: steps 0 .. NB-2 in flight; step 0 retired by every wave before a common
  // barrier, then group 1 falls one barrier behind (its extra barrier pairs with group
  // 0's first mid barrier; group 0 re-aligns after the loop)
#pragma unroll
  for (int t = 0; t < NB - 1; ++t) stage(t);
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(4 * (NB - 2)) : "memory");
  __builtin_amdgcn_s_barrier();
  if (STAG && __builtin_amdgcn_readfirstlane(wr) == 1) __builtin_amdgcn_s_barrier();

  // one K-step (step s of this block): the read section, the mid barrier, the MFMA
  // section (refill first, or -- on a tile's last step, LAST -- after the MFMAs and the
  // tile's residual requests, in the fragment registers the MFMAs free: the epilogue
  // then waits for them and for the two older steps, one round trip per tile and never
  // for the refill, as vmcnt retires in order), the end barrier
  auto kstep = [&](int s, bool LAST, int m0, int n0) {
    read_frags(smem + (s % NB) * BUF);
    // step s+1 retired before the barrier that precedes its reads (NB-3 younger steps
    // of this wave may stay in flight)
    asm volatile("s_waitcnt vmcnt(%0)" ::"n"(4 * (NB - 3)) : "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    if (!LAST) stage(s + NB - 1);  // refill the buffer of step s-1 (read by both groups)
    __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int ks = 0; ks < KS; ++ks)
#pragma unroll
      for (int i = 0; i < FI; ++i)
#pragma unroll
        for (int j = 0; j < FJ; ++j) {
          if constexpr (MF == 16)
            acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bq[ks][j], af[ks][i], acc[i][j], 0, 0, 0);
          else
            acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(bq[ks][j], af[ks][i], acc[i][j], 0, 0, 0);
        }
    __builtin_amdgcn_s_setprio(0);
    if (LAST) {
#pragma unroll
      for (int i = 0; i < FI; ++i) {
        const int gr = m0 + rbase + i * MF + (lane & (MF - 1));
#pragma unroll
        for (int j = 0; j < FJ; ++j)
#pragma unroll
          for (int g = 0; g < AV / 4; ++g) {
            const int col = n0 + cbase + (MF == 16 ? j * 16 + 4 * (lane >> 4) : j * 32 + 8 * g + 4 * (lane >> 5));
            rres[i][j * (AV / 4) + g] =
                gr < M ? *reinterpret_cast<const uint2*>(R + (size_t)gr * ldr + col) : make_uint2(0u, 0u);
          }
      }
      stage(s + NB - 1);
    }
    __builtin_amdgcn_s_barrier();
  };

  int s = 0;
  for (int tile = 0; tile < my_tiles; ++tile) {
    int m0, n0;
    tile_mn((int)blockIdx.x + tile * G, m0, n0);
    zero_acc();
    for (int kt = 0; kt < KT - 1; ++kt, ++s) kstep(s, false, m0, n0);
    kstep(s, true, m0, n0);
    ++s;
    // ---- tile done: epilogue from the accumulators (no barriers), then the next tile.
    // MF 16: lane holds rows rbase + 16i + (lane & 15), columns cbase + 16j + 4·(lane >> 4)
    // + q; MF 32: rows rbase + 32i + (lane & 31), columns cbase + 32j + 8g + 4·(lane >> 5)
    // + q (value 4g + q).  An 8-column x² chunk: its first 4 columns in one lane, its last
    // 4 in the partner lane (xor 16 / xor 32), the fmaf chain run through both in order.
    const bool want_ss = na.ssout != nullptr;
#pragma unroll
    for (int i = 0; i < FI; ++i) {
      const int gr = m0 + rbase + i * MF + (lane & (MF - 1));
      const bool ok = gr < M;
      constexpr int NCH = FJ * (AV / 4);  // this lane's 4-column groups
      float own[NCH];
#pragma unroll
      for (int j = 0; j < FJ; ++j)
#pragma unroll
        for (int g = 0; g < AV / 4; ++g) {
          const int col = n0 + cbase + (MF == 16 ? j * 16 + 4 * (lane >> 4) : j * 32 + 8 * g + 4 * (lane >> 5));
          const uint2 rv = rres[i][j * (AV / 4) + g];
          float o[4];
          const uint32_t rw[2] = {rv.x, rv.y};
#pragma unroll
          for (int q = 0; q < 4; ++q) {
            const float prod = bf2f(f2bf(acc[i][j][4 * g + q]));  // the staged bf16 product (cfg 28's C tile)
            const float res = bf2f((rw[q >> 1] >> ((q & 1) * 16)) & 0xffffu);
            o[q] = bf2f(f2bf(prod + res));
          }
          if (ok)
            *reinterpret_cast<uint2*>(C + (size_t)gr * ldc + col) =
                make_uint2((uint32_t)f2bf(o[0]) | ((uint32_t)f2bf(o[1]) << 16),
                           (uint32_t)f2bf(o[2]) | ((uint32_t)f2bf(o[3]) << 16));
          const float first = fmaf(o[2], o[2], fmaf(o[3], o[3], fmaf(o[0], o[0], fmaf(o[1], o[1], 0.f))));
          const float recv = __shfl_xor(first, MF == 16 ? 16 : 32, 64);
          own[j * (AV / 4) + g] = fmaf(o[2], o[2], fmaf(o[3], o[3], fmaf(o[0], o[0], fmaf(o[1], o[1], recv))));
        }
      if (want_ss) {
        float sum = 0.f;
        if constexpr (MF == 16) {
          // lane group 1 holds chunks 0, 2 .. 10 of the row's 96-column part, group 3
          // chunks 1, 3 .. 11: summed left to right in group 1
          float other[NCH];
#pragma unroll
          for (int c = 0; c < NCH; ++c) other[c] = __shfl_xor(own[c], 32, 64);
#pragma unroll
          for (int c = 0; c < NCH; ++c) {
            sum += own[c];
            sum += other[c];
          }
          if ((lane >> 4) == 1 && ok) na.ssout[(size_t)(n0 / 96 + wj) * na.ld + gr] = sum;
        } else {
          // the upper half-wave holds all 12 chunks of its row, in order
#pragma unroll
          for (int c = 0; c < NCH; ++c) sum += own[c];
          if ((lane >> 5) == 1 && ok) na.ssout[(size_t)(n0 / 96 + wj) * na.ld + gr] = sum;
        }
      }
    }
  }
  if (STAG && __builtin_amdgcn_readfirstlane(wr) == 0) __builtin_amdgcn_s_barrier();  // re-align the groups
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // the tail's dummy DMAs
}

int g_group_m = 8;  // M-tiles per rasterisation group (sg_gemm_set_group_m)

template <int BM, int BN, int WM, int WN, int EPI, int NORM, int ST, int BKT = BK>
int launch(const void* A, int lda, const void* W, void* C, int ldc, const void* R, int ldr, int M, int N, int K,
           float eps, hipStream_t stream, const RopeArgs& ra = RopeArgs{}, const ArgmaxArgs& xa = ArgmaxArgs{},
           const NormArgs& na = NormArgs{}) {
  // the staged C tile must fit in the K-loop buffers (not so for 256-wide plain outputs)
  constexpr int BNO = EPI == 2 ? BN / 2 : BN;
  if constexpr (BM * (BNO + 8) > ST * (BM + BN) * BKT) {
    return -3;
  } else {
    if (K % BKT) return -2;
    const int tm = (M + BM - 1) / BM, tn = N / BN;
    hipLaunchKernelGGL((gemm_fused_kernel<BM, BN, WM, WN, EPI, NORM, ST, 0, BKT>), dim3(tm * tn), dim3(WM * WN * 64), 0,
                       stream, (const uint16_t*)A, lda, (const uint16_t*)W, (uint16_t*)C, ldc, (const uint16_t*)R,
                       ldr, M, N, K, eps, tm, tn, g_group_m > 0 ? g_group_m : 1, ra, xa, na);
    return 0;
  }
}

template <int BM, int BN, int WM, int WN, int ST>
int dispatch_epi(int epi, int norm, const void* A, int lda, const void* W, void* C, int ldc, const void* R, int ldr,
                 int M, int N, int K, float eps, hipStream_t s, const NormArgs& na) {
  const RopeArgs ra{};
  const ArgmaxArgs xa{};
#define SG_L(E, NM) return launch<BM, BN, WM, WN, E, NM, ST>(A, lda, W, C, ldc, R, ldr, M, N, K, eps, s, ra, xa, na)
  if (epi == 0 && norm == 0) SG_L(0, 0);
  if (epi == 0 && norm == 1) SG_L(0, 1);
  if (epi == 1 && norm == 0) SG_L(1, 0);
  if (epi == 2 && norm == 1) SG_L(2, 1);
  if (epi == 2 && norm == 2) SG_L(2, 2);
  if (epi == 2 && norm == 0) SG_L(2, 0);
#undef SG_L
  return -3;
}

// 96 / 192-wide tiles (3 MFMA columns per wave: no SwiGLU pairing) — the N = 576
// residual GEMMs (o-proj, down-proj) and plain stores only
template <int BM, int BN, int WM, int WN, int ST, int BKT = BK>
int dispatch_resid(int epi, int norm, const void* A, int lda, const void* W, void* C, int ldc, const void* R, int ldr,
                   int M, int N, int K, float eps, hipStream_t s, const NormArgs& na) {
  const RopeArgs ra{};
  const ArgmaxArgs xa{};
  if (epi == 1 && norm == 0)
    return launch<BM, BN, WM, WN, 1, 0, ST, BKT>(A, lda, W, C, ldc, R, ldr, M, N, K, eps, s, ra, xa, na);
  if (epi == 0 && norm == 0)
    return launch<BM, BN, WM, WN, 0, 0, ST, BKT>(A, lda, W, C, ldc, R, ldr, M, N, K, eps, s, ra, xa, na);
  if (epi == 0 && norm == 1)
    return launch<BM, BN, WM, WN, 0, 1, ST, BKT>(A, lda, W, C, ldc, R, ldr, M, N, K, eps, s, ra, xa, na);
  return -3;
}

}  // namespace

// Tile configurations: BM x BN (wave grid), pipeline stages.
//   0: 128x128 (2x2) 2st   1: 128x64 (2x2) 2st   2: 64x128 (1x4) 2st   3: 64x64 (2x2) 2st
//   4: 128x64  (2x2) 3st   5: 64x64  (2x2) 3st   6: 64x64  (2x2) 4st   7: 128x128 (2x2) 3st
//   8: 64x128  (1x4) 3st   9: 256x128 (4x2) 2st, 8 waves   10: 256x256 (2x4) 2st, 8 waves
//  11: 128x256 (2x4) 2st, 8 waves   12: 256x64 (4x2) 2st, 8 waves   13: 128x128 (2x4) 2st, 8 waves
//  14: 256x128 (4x2) 3st, 8 waves   15: 128x256 (2x4) 3st, 8 waves   16: 256x64 (4x2) 4st, 8 waves
//  17: 32x64 (2x2) 2st   18: 32x64 (2x2) 4st — small-M decode buckets: twice the tiles of 64x64
//  19: 256x256 (2x4) staggered 8-wave SwiGLU GEMM (gemm256_swiglu_kernel; epi 2 only)
//  20: its persistent form (gemm256p_swiglu_kernel; epi 2 only; NORM 2 needs ss_ld % 4 == 0)
//  21: 128x96 (2x2) 2st   22: 64x96 (2x2) 2st   23: 128x192 (2x4) 2st, 8 waves
//  24: 256x96 (4x2) 2st, 8 waves   25: 128x96 (2x2) 3st   26: 64x192 (1x4) 2st
//  27: 32x96 (2x2) 2st — small-M form of 21 / 22 (the same 96-wide N tiling at every M)
//      (21..27: epi 0 / 1 only — 48-wide wave tiles for the N = 576 residual GEMMs)
//  28: 128x192 (2x2) 2st   29: 256x96 (4x1) 2st — 64x96 wave tiles
//  30: 128x96 (4x2) 2st, 8 waves   31: 64x96 (4x2) 2st, 8 waves
//  32: 256x192 (4x2) 2st, 8 waves — 64x96 wave tiles (epi 0 / 1 only)
//  33: 128x192 (2x2) BK 32, 4st   34: 256x192 (4x2) BK 32, 4st, 8 waves (epi 0 / 1 only)
//  35: 256x192 persistent staggered residual GEMM (gemm256p_resid_kernel, 4 ring buffers,
//      16x16x32 MFMAs; epi 1 only)   36: 35 without the group stagger (A/B)   37: 35 with
//      32x32x16 MFMAs   38: 37 with 5 ring buffers
//  42: 20 with both A register sets (no p4 LDS re-read; A/B)
//  39: (QKV+RoPE only, sg_gemm_qkv_rope) q / k heads through the persistent staggered
//      256x256 QK+RoPE kernel (gemm256p_qk_rope_kernel), v heads through 28; 40 / 41: its
//      q / k part / v part alone (timing A/B only: partial outputs)
// Returns 0, or <0 on a shape the kernel does not cover (the launch is then
// skipped — the Python wrapper raises).
extern "C" {

void sg_gemm_set_group_m(int gm) { g_group_m = gm; }

// Timing probe: the 128x128 SwiGLU+norm GEMM (cfg 0) with its K loop reduced to
// loads only (mode 1) or MFMAs only (mode 2); mode 0 = the real kernel.
int sg_gemm_probe(const void* A, const void* W, void* C, int M, int N, int K, int mode, hipStream_t stream) {
  const int tm = (M + 127) / 128, tn = N / 128;
  if (K % BK || N % 128) return -2;
#define SG_PROBE(MODE)                                                                                          \
  hipLaunchKernelGGL((gemm_fused_kernel<128, 128, 2, 2, 2, 1, 2, MODE>), dim3(tm * tn), dim3(256), 0, stream, \
                     (const uint16_t*)A, K, (const uint16_t*)W, (uint16_t*)C, N / 2, nullptr, 0, M, N, K, 1e-5f, tm, \
                     tn, g_group_m, RopeArgs{}, ArgmaxArgs{}, NormArgs{})
  if (mode == 1) SG_PROBE(1);
  else if (mode == 2) SG_PROBE(2);
  else if (mode == 3) SG_PROBE(3);
  else if (mode == 4) SG_PROBE(4);
  else SG_PROBE(0);
#undef SG_PROBE
  return 0;
}

// norm: 0 none, 1 in-kernel row scale, 2 row scale from ssin ([16][ss_ld] x² partials,
// zero-padded); ssout (EPI 1 only, may be null): this GEMM's output-row partials.
int sg_gemm(const void* A, int lda, const void* W, void* C, int ldc, const void* R, int ldr, int M, int N, int K,
            int epi, int norm, float eps, int cfg, const float* ssin, float* ssout, int ss_ld, hipStream_t stream) {
  static const int BNs[39] = {128, 64, 128, 64, 64, 64, 64, 128, 128, 128, 256, 256, 64, 128, 128, 256, 64, 64, 64,
                             256, 256, 96, 96, 192, 96, 96, 192, 96, 192, 96, 96, 96, 192, 192, 192, 192, 192,
                             192, 192};
  const bool twoa = cfg == 42;  // A/B form of 20
  if (twoa) cfg = 20;
  if (cfg < 0 || cfg > 38) return -1;
  if (M <= 0 || K % BK != 0 || N % BNs[cfg] != 0 || lda % 8 != 0 || ldc % 8 != 0 || (R && ldr % 8 != 0)) return -2;
  if (epi == 1 && !R) return -2;
  if ((norm == 2 && (!ssin || ss_ld < M)) || (ssout && (epi != 1 || N / BNs[cfg] > SS_PARTS || ss_ld < M)))
    return -2;
  const NormArgs na{ssin, ssout, ss_ld};
  if (cfg == 19) {  // 256x256 staggered 8-wave SwiGLU GEMM
    if (epi != 2) return -3;
    const int tm = (M + 255) / 256, tn = N / 256;
    const int gmv = g_group_m > 0 ? g_group_m : 1;
#define SG_256(NM)                                                                                                  \
  hipLaunchKernelGGL((gemm256_swiglu_kernel<NM>), dim3(tm * tn), dim3(512), 0, stream, (const uint16_t*)A, lda,   \
                     (const uint16_t*)W, (uint16_t*)C, ldc, M, N, K, eps, tm, tn, gmv, na)
    if (norm == 2) SG_256(2);
    else if (norm == 1) SG_256(1);
    else SG_256(0);
#undef SG_256
    return 0;
  }
  if (cfg == 20) {  // persistent form: one block per CU (256 CUs), tiles overlapped
    if (epi != 2) return -3;
    if (norm == 2 && ss_ld % 4 != 0) return -2;
    const int tm = (M + 255) / 256, tn = N / 256, T = tm * tn;
    const int grid = T < 256 ? T : 256;
    const int gmv = g_group_m > 0 ? g_group_m : 1;
#define SG_256P(...)                                                                                                  \
  hipLaunchKernelGGL((gemm256p_swiglu_kernel<__VA_ARGS__>), dim3(grid), dim3(512), 0, stream, (const uint16_t*)A, lda,       \
                     (const uint16_t*)W, (uint16_t*)C, ldc, M, N, K, eps, tm, tn, gmv, na)
    if (twoa) {
      if (norm == 2) SG_256P(2, true);
      else if (norm == 1) SG_256P(1, true);
      else SG_256P(0, true);
    } else if (norm == 2) SG_256P(2);
    else if (norm == 1) SG_256P(1);
    else SG_256P(0);
#undef SG_256P
    return 0;
  }
  if (cfg >= 35 && cfg <= 38) {  // persistent staggered residual GEMM: one block per CU
    if (epi != 1 || norm != 0 || K % 32 != 0) return -3;
    if (ssout && N / 96 > SS_PARTS) return -2;
    const int tm = (M + 255) / 256, tn = N / 192, T = tm * tn;
    const int grid = T < 256 ? T : 256;
    const int gmv = g_group_m > 0 ? g_group_m : 1;
#define SG_RP(NB_, MF_, ...)                                                                                  \
  hipLaunchKernelGGL((gemm256p_resid_kernel<NB_, MF_, ##__VA_ARGS__>), dim3(grid), dim3(512), 0, stream, (const uint16_t*)A, lda, \
                     (const uint16_t*)W, (uint16_t*)C, ldc, (const uint16_t*)R, ldr, M, N, K, tm, tn, gmv, na)
    if (cfg == 35) SG_RP(4, 16);
    else if (cfg == 36) SG_RP(4, 16, false);  // A/B: the same loop without the group stagger
    else if (cfg == 37) SG_RP(4, 32);
    else SG_RP(5, 32);
#undef SG_RP
    return 0;
  }
#define SG_ARGS epi, norm, A, lda, W, C, ldc, R, ldr, M, N, K, eps, stream, na
  switch (cfg) {
    case 0: return dispatch_epi<128, 128, 2, 2, 2>(SG_ARGS);
    case 1: return dispatch_epi<128, 64, 2, 2, 2>(SG_ARGS);
    case 2: return dispatch_epi<64, 128, 1, 4, 2>(SG_ARGS);
    case 3: return dispatch_epi<64, 64, 2, 2, 2>(SG_ARGS);
    case 4: return dispatch_epi<128, 64, 2, 2, 3>(SG_ARGS);
    case 5: return dispatch_epi<64, 64, 2, 2, 3>(SG_ARGS);
    case 6: return dispatch_epi<64, 64, 2, 2, 4>(SG_ARGS);
    case 7: return dispatch_epi<128, 128, 2, 2, 3>(SG_ARGS);
    case 8: return dispatch_epi<64, 128, 1, 4, 3>(SG_ARGS);
    case 9: return dispatch_epi<256, 128, 4, 2, 2>(SG_ARGS);
    case 10: return dispatch_epi<256, 256, 2, 4, 2>(SG_ARGS);
    case 11: return dispatch_epi<128, 256, 2, 4, 2>(SG_ARGS);
    case 12: return dispatch_epi<256, 64, 4, 2, 2>(SG_ARGS);
    case 13: return dispatch_epi<128, 128, 2, 4, 2>(SG_ARGS);
    case 14: return dispatch_epi<256, 128, 4, 2, 3>(SG_ARGS);
    case 15: return dispatch_epi<128, 256, 2, 4, 3>(SG_ARGS);
    case 16: return dispatch_epi<256, 64, 4, 2, 4>(SG_ARGS);
    case 17: return dispatch_epi<32, 64, 2, 2, 2>(SG_ARGS);
    case 18: return dispatch_epi<32, 64, 2, 2, 4>(SG_ARGS);
    case 21: return dispatch_resid<128, 96, 2, 2, 2>(SG_ARGS);
    case 22: return dispatch_resid<64, 96, 2, 2, 2>(SG_ARGS);
    case 23: return dispatch_resid<128, 192, 2, 4, 2>(SG_ARGS);
    case 24: return dispatch_resid<256, 96, 4, 2, 2>(SG_ARGS);
    case 25: return dispatch_resid<128, 96, 2, 2, 3>(SG_ARGS);
    case 26: return dispatch_resid<64, 192, 1, 4, 2>(SG_ARGS);
    // 64x96 wave tiles (4 waves): 10 fragment reads per 24 MFMAs and (BM + BN) / (BM * BN)
    // staged bytes per output 28 % below the 64x48 wave tiles of 21 / 23 / 24 (LDS-bound loop)
    case 28: return dispatch_resid<128, 192, 2, 2, 2>(SG_ARGS);
    case 29: return dispatch_resid<256, 96, 4, 1, 2>(SG_ARGS);
    // 8 waves on the 96-wide tiles (32x48 / 16x48 wave tiles): twice the waves per CU to
    // hide the one-tile-per-block latency of the short K loops (K = 576 / 1536)
    case 30: return dispatch_resid<128, 96, 4, 2, 2>(SG_ARGS);
    case 31: return dispatch_resid<64, 96, 4, 2, 2>(SG_ARGS);
    // 256x192, 8 waves, the 64x96 wave tiles of 28: 1.4x its MFMA work per staged byte
    // (the big-M residual loop is L2-bound at 77 FLOP/B; this tile is 110)
    case 32: return dispatch_resid<256, 192, 4, 2, 2>(SG_ARGS);
    // BK 32 with 4 stages in the same LDS: three K-steps of loads in flight instead of one
    // (the residual loop waits on loads: bytes in flight per CU set its rate)
    case 33: return dispatch_resid<128, 192, 2, 2, 4, 32>(SG_ARGS);
    case 34: return dispatch_resid<256, 192, 4, 2, 4, 32>(SG_ARGS);
    default: return dispatch_resid<32, 96, 2, 2, 2>(SG_ARGS);
  }
#undef SG_ARGS
}

// QKV projection with the RMSNorm prologue and the RoPE + KV-cache epilogue
// (replaces gemm + sg_rope_qkv_cache).  W: [(nh + 2 nkv)·64, K], norm folded in.
// cfg must have BN = 64 (1, 3, 5, 17 or 18) or 192 (23: 128x192 8 waves, 28: 4 waves, 26: 64x192; three
// heads per N tile, so nh and nkv must be multiples of 3).
// ssin non-null: the row scales come from the producer's partials (NORM 2).
int sg_gemm_qkv_rope(const void* A, int lda, const void* W, int M, int K, float eps, int cfg, const int* pos,
                     const int* slot, const void* cos_sin, void* q_out, void* k_cache, void* vt_cache, int nh, int nkv,
                     int Lmax, int p0, const float* ssin, int ss_ld, hipStream_t stream) {
  const int N = (nh + 2 * nkv) * 64;
  if (M <= 0 || K % BK != 0 || lda % 8 != 0 || (Lmax % 8) != 0) return -2;
  RopeArgs ra{pos, slot, (const float2*)cos_sin, (uint16_t*)q_out, (uint16_t*)k_cache, (uint16_t*)vt_cache,
              nh, nkv, Lmax, p0};
  if (ssin && ss_ld < M) return -2;
  const NormArgs na{ssin, nullptr, ss_ld};
  const ArgmaxArgs xa{};
#define SG_QKV(BM_, ST_)                                                                                              \
  return ssin ? launch<BM_, 64, 2, 2, 3, 2, ST_>(A, lda, W, nullptr, 64, nullptr, 0, M, N, K, eps, stream, ra, xa, na) \
              : launch<BM_, 64, 2, 2, 3, 1, ST_>(A, lda, W, nullptr, 64, nullptr, 0, M, N, K, eps, stream, ra, xa, na)
  switch (cfg) {
    case 1: SG_QKV(128, 2);
    case 3: SG_QKV(64, 2);
    case 5: SG_QKV(64, 3);
    case 17: SG_QKV(32, 2);
    case 18: SG_QKV(32, 4);
    case 23:
      if (nh % 3 || nkv % 3) return -2;
      return ssin ? launch<128, 192, 2, 4, 3, 2, 2>(A, lda, W, nullptr, 64, nullptr, 0, M, N, K, eps, stream, ra, xa, na)
                  : launch<128, 192, 2, 4, 3, 1, 2>(A, lda, W, nullptr, 64, nullptr, 0, M, N, K, eps, stream, ra, xa, na);
    case 26:
      if (nh % 3 || nkv % 3) return -2;
      return ssin ? launch<64, 192, 1, 4, 3, 2, 2>(A, lda, W, nullptr, 64, nullptr, 0, M, N, K, eps, stream, ra, xa, na)
                  : launch<64, 192, 1, 4, 3, 1, 2>(A, lda, W, nullptr, 64, nullptr, 0, M, N, K, eps, stream, ra, xa, na);
    case 28:  // 128x192, 4 waves: 64x96 wave tiles
      if (nh % 3 || nkv % 3) return -2;
      return ssin ? launch<128, 192, 2, 2, 3, 2, 2>(A, lda, W, nullptr, 64, nullptr, 0, M, N, K, eps, stream, ra, xa, na)
                  : launch<128, 192, 2, 2, 3, 1, 2>(A, lda, W, nullptr, 64, nullptr, 0, M, N, K, eps, stream, ra, xa, na);
    case 39:    // q, k heads: persistent staggered 256x256 QK+RoPE kernel; v heads: cfg 28
    case 40:    // (timing A/B: the q, k part alone)
    case 41: {  // (timing A/B: the v part alone)
      if (nh % 3 || nkv % 3 || (nh + nkv) % 4 || (ssin && ss_ld % 4 != 0)) return -2;
      const int Nqk = (nh + nkv) * 64, tm = (M + 255) / 256, tn = Nqk / 256, T = tm * tn;
      const int grid = T < 256 ? T : 256, gmv = g_group_m > 0 ? g_group_m : 1;
      if (cfg == 41) {
      } else if (ssin)
        hipLaunchKernelGGL((gemm256p_qk_rope_kernel<2>), dim3(grid), dim3(512), 0, stream, (const uint16_t*)A, lda,
                           (const uint16_t*)W, M, Nqk, K, eps, tm, tn, gmv, na, ra);
      else
        hipLaunchKernelGGL((gemm256p_qk_rope_kernel<1>), dim3(grid), dim3(512), 0, stream, (const uint16_t*)A, lda,
                           (const uint16_t*)W, M, Nqk, K, eps, tm, tn, gmv, na, ra);
      if (cfg == 40) return 0;
      RopeArgs rv = ra;
      rv.hb = nh + nkv;
      const uint16_t* Wv = (const uint16_t*)W + (size_t)Nqk * K;
      return ssin ? launch<128, 192, 2, 2, 3, 2, 2>(A, lda, Wv, nullptr, 64, nullptr, 0, M, nkv * 64, K, eps, stream, rv, xa, na)
                  : launch<128, 192, 2, 2, 3, 1, 2>(A, lda, Wv, nullptr, 64, nullptr, 0, M, nkv * 64, K, eps, stream, rv, xa, na);
    }
    default: return -1;
  }
#undef SG_QKV
}

// lm_head + FSM-masked arg-max (EPI 4): W [N, K] with the final norm folded in,
// best [M] uint64 zeroed before the launch; cfg 0 (128x128), 3 (64x64), 17 (32x64).
int sg_gemm_argmax(const void* A, int lda, const void* W, int M, int N, int K, float eps, int norm, int cfg,
                   const int* row_state, const int* state_mask, const void* masks, void* best, const float* ssin,
                   int ss_ld, const int* copy_kind, const void* row_masks, hipStream_t stream) {
  if (M <= 0 || K % BK != 0 || lda % 8 != 0 || N % 128 != 0) return -2;
  if (norm == 2 && (!ssin || ss_ld < M)) return -2;
  if (copy_kind != nullptr && row_masks == nullptr) return -2;
  ArgmaxArgs xa{row_state, state_mask, (const uint32_t*)masks, (unsigned long long*)best, copy_kind,
                (const uint32_t*)row_masks};
  RopeArgs ra{};
  const NormArgs na{ssin, nullptr, ss_ld};
#define SG_AM(BM_, BN_, WM_, WN_)                                                                                      \
  return norm == 2 ? launch<BM_, BN_, WM_, WN_, 4, 2, 2>(A, lda, W, nullptr, 8, nullptr, 0, M, N, K, eps, stream, ra, xa, na) \
       : norm      ? launch<BM_, BN_, WM_, WN_, 4, 1, 2>(A, lda, W, nullptr, 8, nullptr, 0, M, N, K, eps, stream, ra, xa, na) \
                   : launch<BM_, BN_, WM_, WN_, 4, 0, 2>(A, lda, W, nullptr, 8, nullptr, 0, M, N, K, eps, stream, ra, xa, na)
  switch (cfg) {
    case 0: SG_AM(128, 128, 2, 2);
    case 3: SG_AM(64, 64, 2, 2);
    case 17: SG_AM(32, 64, 2, 2);
    default: return -1;
  }
#undef SG_AM
}

}  // extern "C"
