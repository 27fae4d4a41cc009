// smsgate_amd — speculative decoding for the schema-constrained extractor (gfx950).
//
// The extractor writes every copied field value with the SMS body's own tokens
// (models/tokenizer.py value_span_ids), so the body is an exact draft source:
// "prompt lookup" drafting.  One speculative step of a decode bucket of B rows:
//
//   sg_spec_plan    three launches.  draft (one thread per row): look up the row's
//                   last token (bigram with the one before, else unigram) in its
//                   body tokens and draft up to K following body tokens, walking
//                   the schema FSM (a delimiter token -- ',' / '&#' / ';' -- is
//                   drafted as <sep>; policy 1 adds forced tokens, implicit value
//                   ends and field-start resumption).  scan (one block): finished
//                   rows take no pseudo-row, the live rows' drafts are water-filled
//                   into the budget T_cap - live rows and packed by an exclusive
//                   scan.  fill (one thread per row): pseudo-row = one query token
//                   at its own position in its row's KV slot; the unused tail
//                   points at a scratch slot and is marked done.
//   verify forward  the decode GEMMs + QKV/RoPE/KV-write run over the T_cap
//                   pseudo-rows; attention is attn_spec_kernel (one wave per row and
//                   kv head, the row's keys read once for all its drafts); the
//                   lm_head GEMM reduces each pseudo-row to its FSM-masked arg-max
//                   key (sg_gemm_argmax, masked with the state the row would be in
//                   if the drafts before it are accepted).
//   sg_spec_verify_keys  one thread per row: accept drafts while the arg-max equals
//                   the next draft; every arg-max taken is emitted, so a step emits
//                   accepted + 1 tokens.  KV entries written for rejected drafts lie
//                   beyond the row's new position and are overwritten later.
//
// Greedy outputs are bit-identical to one-token decode: every query token runs
// the same per-column arithmetic (tests/test_spec_gpu.py, test_kernels_gpu.py).
#include <hip/hip_runtime.h>
#include <stdint.h>

#define SPEC_THREADS 1024
#define SPEC_MAX_K 8

static __device__ __forceinline__ float sp_bf2f(uint16_t v) { return __uint_as_float(((uint32_t)v) << 16); }

// Schema-FSM tables (serving/fsm.py), as fsm_sample_kernel reads them.
struct FsmTables {
  const uint32_t* masks;
  const int* state_mask;
  const int* next_sep;
  const int* next_tok;
  const int* enum_tok;
  const int* enum_next;
  int E, sep_token, done_state, V;
};

// next state after emitting `tok` in state `s` (-1 = not allowed / dead end)
static __device__ __forceinline__ int fsm_next(const FsmTables& f, int s, int tok) {
  if (tok == f.sep_token) return f.next_sep[s];
  int ns = f.next_tok[s];
  if (f.E > 0 && ns == -2) {
    ns = -1;
    for (int e = 0; e < f.E; ++e)
      if (f.enum_tok[s * f.E + e] == tok) { ns = f.enum_next[s * f.E + e]; break; }
  }
  return ns;
}

static __device__ __forceinline__ bool fsm_allows(const FsmTables& f, int s, int tok) {
  const uint32_t* m = f.masks + (size_t)f.state_mask[s] * (f.V >> 5);
  return (m[tok >> 5] >> (tok & 31)) & 1u;
}

// token of an arg-max key written by sg_gemm_argmax (0 = nothing allowed -> <sep>)
static __device__ __forceinline__ int key_token(unsigned long long key, int sep_token) {
  return key ? (int)(0xFFFFFFFFu - (uint32_t)(key & 0xFFFFFFFFull)) : sep_token;
}

// ---------------------------------------------------------------------------
// plan, three launches (one thread per row; the scan is the only single-block part):
//   draft  — per row: prompt-lookup drafts (FSM-checked), unclamped count
//   scan   — one block: exclusive scan of the counts, clamp to the draft budget
//   fill   — per row: write the pseudo-rows; then the unused tail
// ---------------------------------------------------------------------------
// first body position (bigram (prev, t), else unigram t) of `t`; -1 if absent
static __device__ __forceinline__ int body_anchor(const int* body, int bl, int t, int prev) {
  if (prev >= 0)
    for (int q = 1; q < bl; ++q)
      if (body[q] == t && body[q - 1] == prev) return q;
  for (int q = 0; q < bl; ++q)
    if (body[q] == t) return q;
  return -1;
}

// policy 0 (round-2 first cut): copy the body after the last token's anchor, stop at
//   the first <sep> or schema-forbidden token; nothing at a field start.
// policy 1: (a) tokens the schema forces (the only allowed token of the state, e.g.
//   the rest of an enum value or the <sep> after a full field) are drafted first;
//   (b) a body token the field forbids where <sep> is allowed ends the value
//   implicitly (<sep>, then the token starts the next field: "1500.00 RUB");
//   (c) the copy runs on past <sep> into the next field; (d) at a field start
//   (last token <sep>) the copy resumes after the previous value's last token.
// scripts/spec_sim.py replays gold answers through both (14.9 -> 11.8 steps/message).
__global__ void __launch_bounds__(256) spec_draft_kernel(
    FsmTables fsm, const int* __restrict__ state, int B, int K, int sep_token, const int* __restrict__ tok_buf,
    const int* __restrict__ slot, const int* __restrict__ done, const int* __restrict__ out_buf,
    const int* __restrict__ out_len, int max_out, const int* __restrict__ body_buf, const int* __restrict__ body_len,
    int LB, const uint8_t* __restrict__ delim, const int* __restrict__ forced, int policy,
    int* __restrict__ draft_buf, int* __restrict__ row_nd) {
  const int r = blockIdx.x * blockDim.x + threadIdx.x;
  if (r >= B) return;
  int n = 0;
  int* dr = draft_buf + r * SPEC_MAX_K;
  if (!done[r]) {
    const int len = out_len[r];
    const int* ob = out_buf + (size_t)r * max_out;
    // t1 = last token, t2 / t3 the ones before it (-1 = none)
    int t1 = tok_buf[r], t2 = len >= 2 ? ob[len - 2] : -1, t3 = len >= 3 ? ob[len - 3] : -1;
    int s = state[r];
    if (policy >= 1) {
      while (n < K && s != fsm.done_state && forced[s] >= 0) {
        const int x = forced[s];
        dr[n++] = x;
        s = fsm_next(fsm, s, x);
        t3 = t2;
        t2 = t1;
        t1 = x;
        if (s < 0) break;
      }
    }
    const int sl = slot[r];
    const int* body = body_buf + (size_t)sl * LB;
    const int bl = body_len[sl];
    int j = -1;
    if (s >= 0 && s != fsm.done_state && n < K) {
      if (t1 != sep_token) {
        j = body_anchor(body, bl, t1, t2 == sep_token ? -1 : t2);
      } else if (policy >= 1 && t2 >= 0 && t2 != sep_token) {
        j = body_anchor(body, bl, t2, t3 == sep_token ? -1 : t3);
        if (j >= 0) {
          while (j + 1 < bl && delim[body[j + 1]]) ++j;  // the delimiter that ended the value
        }
      }
    }
    if (j >= 0) {
      // walk the schema FSM along the draft: a token the FSM forbids can never be
      // accepted (the verify arg-max is masked), so the draft stops before it
      for (int q = j + 1; q < bl && n < K;) {
        const int x = delim[body[q]] ? sep_token : body[q];
        if (!fsm_allows(fsm, s, x)) {
          if (policy >= 1 && x != sep_token && fsm_allows(fsm, s, sep_token)) {
            dr[n++] = sep_token;  // implicit end of the value; x starts the next field
            s = fsm_next(fsm, s, sep_token);
            if (s < 0 || s == fsm.done_state || !fsm_allows(fsm, s, x)) break;
            continue;
          }
          break;
        }
        const int ns = fsm_next(fsm, s, x);
        if (ns < 0) break;
        dr[n++] = x;
        s = ns;
        ++q;
        if (ns == fsm.done_state || (policy == 0 && x == sep_token)) break;
      }
    }
  }
  row_nd[r] = done[r] ? -1 : n;  // -1: finished row, no pseudo-row at all
}

// block-wide exclusive scan of one int per thread (all SPEC_THREADS threads call it)
static __device__ __forceinline__ int block_excl_scan(int v, int* wsum, int& total) {
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  constexpr int NWV = SPEC_THREADS / 64;
  int incl = v;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const int u = __shfl_up(incl, o, 64);
    if (lane >= o) incl += u;
  }
  if (lane == 63) wsum[wid] = incl;
  __syncthreads();
  if (tid == 0) {
    int acc = 0;
    for (int w = 0; w < NWV; ++w) {
      const int x = wsum[w];
      wsum[w] = acc;
      acc += x;
    }
    wsum[NWV] = acc;
  }
  __syncthreads();
  const int res = wsum[wid] + incl - v;
  total = wsum[NWV];
  __syncthreads();  // wsum is reused by the next call
  return res;
}

// one block: finished rows (row_nd = -1) get no pseudo-row, so the budget is
// D_cap = T_cap - live rows; the live rows' draft counts are clamped to it by water
// filling -- every row keeps min(nd, c) drafts for the largest cap c that fits, the
// rest of the budget gives one more draft to the first rows with nd > c -- so the
// budget goes to the early (most likely accepted) drafts of as many rows as
// possible; then row_start[r] = pseudo-rows of rows < r; meta[0] = pseudo-rows used.
__global__ void __launch_bounds__(SPEC_THREADS) spec_scan_kernel(int B, int K, int T_cap, int* __restrict__ row_start,
                                                                 int* __restrict__ row_nd, int* __restrict__ meta) {
  __shared__ int wsum[SPEC_THREADS / 64 + 1];
  __shared__ int tot[SPEC_MAX_K + 1];
  __shared__ int s_c, s_extra;
  const int tid = threadIdx.x, lane = tid & 63;
  const int RPT = (B + SPEC_THREADS - 1) / SPEC_THREADS;
  const int r0 = tid * RPT, r1 = min(B, r0 + RPT);
  if (tid <= SPEC_MAX_K) tot[tid] = 0;
  __syncthreads();
  {
    int live = 0;
    for (int r = r0; r < r1; ++r) live += row_nd[r] >= 0;
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) live += __shfl_xor(live, o, 64);
    if (lane == 0) atomicAdd(&tot[0], live);  // LDS atomic; tot[0] = live rows until read below
  }
  __syncthreads();
  const int D_cap = T_cap - tot[0];
  __syncthreads();
  if (tid == 0) tot[0] = 0;
  // tot[c] = sum over rows of min(nd, c)
  for (int c = 1; c <= K; ++c) {
    int part = 0;
    for (int r = r0; r < r1; ++r) part += min(max(row_nd[r], 0), c);
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) part += __shfl_xor(part, o, 64);
    if (lane == 0) atomicAdd(&tot[c], part);  // LDS atomic
  }
  __syncthreads();
  if (tid == 0) {
    int c = 0;
    for (int cc = 1; cc <= K; ++cc)
      if (tot[cc] <= D_cap) c = cc;
    s_c = c;
    s_extra = D_cap - tot[c];
  }
  __syncthreads();
  const int c = s_c, extra = s_extra;
  int over = 0;
  for (int r = r0; r < r1; ++r) over += row_nd[r] > c;
  int total;
  int rank = block_excl_scan(over, wsum, total);
  int mine = 0;
  for (int r = r0; r < r1; ++r) {
    const int n = row_nd[r];
    if (n < 0) continue;  // finished: stays -1
    int f = min(n, c);
    if (n > c) {
      f += rank < extra;
      ++rank;
    }
    row_nd[r] = f;
    mine += 1 + f;
  }
  int dstart = block_excl_scan(mine, wsum, total);
  for (int r = r0; r < r1; ++r) {
    row_start[r] = dstart;
    dstart += 1 + row_nd[r];  // + 0 for a finished row
  }
  if (tid == 0) meta[0] = total;
}

__global__ void __launch_bounds__(256) spec_fill_kernel(
    FsmTables fsm, const int* __restrict__ state, int B, int T_cap, int scratch_slot, const int* __restrict__ tok_buf,
    const int* __restrict__ pos, const int* __restrict__ slot, const int* __restrict__ done,
    const int* __restrict__ draft_buf, const int* __restrict__ row_start, const int* __restrict__ row_nd,
    const int* __restrict__ meta, int* __restrict__ x_tok, int* __restrict__ x_pos, int* __restrict__ x_slot,
    int* __restrict__ x_done, int* __restrict__ x_state) {
  const int g = blockIdx.x * blockDim.x + threadIdx.x;
  if (g < B && row_nd[g] >= 0) {  // a finished row (row_nd = -1) has no pseudo-row
    const int r = g, st = row_start[r], nc = row_nd[r];
    const int p = pos[r], sl = slot[r], dn = done[r];
    int s = state[r];
    x_tok[st] = tok_buf[r];
    x_pos[st] = p;
    x_slot[st] = sl;
    x_done[st] = dn;
    x_state[st] = dn ? fsm.done_state : s;
    for (int i = 0; i < nc; ++i) {
      const int x = draft_buf[r * SPEC_MAX_K + i];
      s = fsm_next(fsm, s, x);  // valid: the draft walk checked it
      x_tok[st + 1 + i] = x;
      x_pos[st + 1 + i] = p + 1 + i;
      x_slot[st + 1 + i] = sl;
      x_done[st + 1 + i] = 0;
      x_state[st + 1 + i] = s;  // the state the row is in IF drafts 0..i are accepted
    }
  }
  // unused tail: scratch slot, position 0, skipped by attention
  const int used = meta[0];
  for (int i = used + g; i < T_cap; i += gridDim.x * blockDim.x) {
    x_tok[i] = 0;
    x_pos[i] = 0;
    x_slot[i] = scratch_slot;
    x_done[i] = 1;
    x_state[i] = fsm.done_state;
  }
}

// ---------------------------------------------------------------------------
// verify from arg-max keys (sg_gemm_argmax already masked each pseudo-row with
// x_state): one thread per row, no logits read.
// ---------------------------------------------------------------------------
// the greedy verification of row b (spec_verify_keys_kernel); returns the tokens emitted
static __device__ __forceinline__ int spec_verify_row(
    const FsmTables& fsm, const unsigned long long* __restrict__ best, int* __restrict__ state, int* __restrict__ tok_buf,
    int* __restrict__ out_buf, int* __restrict__ out_len, int* __restrict__ done, int* __restrict__ pos,
    const int* __restrict__ x_tok, const int* __restrict__ row_start, const int* __restrict__ row_nd, int max_out,
    int b) {
  const int st = row_start[b], nd = row_nd[b];
  int s = state[b], len = out_len[b], p = pos[b], emitted = 0, tok = tok_buf[b];
  bool fin = false;
  for (int i = 0; i <= nd; ++i) {
    tok = key_token(best[st + i], fsm.sep_token);
    const int ns = fsm_next(fsm, s, tok);
    out_buf[(size_t)b * max_out + len] = tok;
    ++len;
    ++emitted;
    s = ns < 0 ? fsm.done_state : ns;
    if (ns < 0 || ns == fsm.done_state || len >= max_out) {
      fin = true;
      break;
    }
    ++p;
    if (!(i < nd && tok == x_tok[st + i + 1])) break;
  }
  out_len[b] = len;
  tok_buf[b] = tok;
  state[b] = s;
  pos[b] = p;
  if (fin) done[b] = 1;
  return emitted;
}

__global__ void __launch_bounds__(256) spec_verify_keys_kernel(
    FsmTables fsm, const unsigned long long* __restrict__ best, int* __restrict__ state, int* __restrict__ tok_buf,
    int* __restrict__ out_buf, int* __restrict__ out_len, int* __restrict__ done, int* __restrict__ pos,
    const int* __restrict__ x_tok, const int* __restrict__ row_start, const int* __restrict__ row_nd,
    int* __restrict__ accepted, int max_out, int B, unsigned long long* __restrict__ counts) {
  const int b = blockIdx.x * blockDim.x + threadIdx.x;
  // counts (optional): [tokens emitted, live rows] of this step, summed per wave and added
  // with one atomic per wave (the engine's spec_stats; was four torch kernels per step)
  int emitted = 0;
  if (b < B && !done[b]) emitted = spec_verify_row(fsm, best, state, tok_buf, out_buf, out_len, done, pos, x_tok,
                                                   row_start, row_nd, max_out, b);
  if (b < B && accepted != nullptr) accepted[b] = emitted;
  if (counts != nullptr) {
    unsigned long long e = (unsigned long long)emitted, live = emitted > 0 ? 1ull : 0ull;
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
      e += __shfl_xor(e, o, 64);
      live += __shfl_xor(live, o, 64);
    }
    if ((threadIdx.x & 63) == 0 && e) {
      atomicAdd(&counts[0], e);
      atomicAdd(&counts[1], live);
    }
  }
}


// ---------------------------------------------------------------------------
// one-token decode / prefill sampling from arg-max keys: the FSM step of
// fsm_sample_kernel's greedy path.  Key row i updates state row row_map[i] (or i).
// ---------------------------------------------------------------------------
__global__ void __launch_bounds__(256) fsm_commit_kernel(
    FsmTables fsm, const unsigned long long* __restrict__ best, const int* __restrict__ row_map,
    int* __restrict__ state, int* __restrict__ tok_io, int* __restrict__ out_buf, int* __restrict__ out_len,
    int* __restrict__ done, int* __restrict__ pos, int max_out, int B) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= B) return;
  const int b = row_map ? row_map[i] : i;
  if (done[b]) return;
  const int s = state[b];
  const int tok = key_token(best[i], fsm.sep_token);
  const int ns = fsm_next(fsm, s, tok);
  const int len = out_len[b];
  out_buf[(size_t)b * max_out + len] = tok;
  out_len[b] = len + 1;
  tok_io[b] = tok;
  state[b] = ns < 0 ? fsm.done_state : ns;
  if (ns < 0 || ns == fsm.done_state || len + 1 >= max_out) done[b] = 1;
  else pos[b] = pos[b] + 1;
}

// ---------------------------------------------------------------------------
// span-pointer format: fsm_commit that writes the answer in COPY format.  A start
// pointer is only held (tok_io: the next step's input, and the end state's `prev`);
// the end pointer appends the body tokens start..end and <sep>; <sep> and enum
// tokens are appended as they are.  So out_buf / out_len look exactly like a
// copy-format decode's and everything downstream (harvest, remote clients'
// detokenisation) is unchanged.  Key row i updates state row row_map[i] (or i);
// row_slot[i] is that row's KV slot (its prompt in body_buf).
// ---------------------------------------------------------------------------
__global__ void __launch_bounds__(256) span_commit_kernel(
    FsmTables fsm, const int* __restrict__ copy_kind, const unsigned long long* __restrict__ best,
    const int* __restrict__ row_map, const int* __restrict__ row_slot, const int* __restrict__ body_buf,
    const int* __restrict__ body_len, int LB, int ptr0, int* __restrict__ state, int* __restrict__ tok_io,
    int* __restrict__ out_buf, int* __restrict__ out_len, int* __restrict__ done, int* __restrict__ pos,
    int max_out, int B) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= B) return;
  const int b = row_map ? row_map[i] : i;
  if (done[b]) return;
  const int s = state[b];
  const int tok = key_token(best[i], fsm.sep_token);
  const int ns = fsm_next(fsm, s, tok);
  const int k8 = copy_kind[s] & 0xff;
  int len = out_len[b];
  int* ob = out_buf + (size_t)b * max_out;
  if (k8 == 4) {
    const int sl = row_slot[i];
    const int nb = min(body_len[sl], LB) - 1;
    const int* body = body_buf + (size_t)sl * LB;
    const int s0 = max(0, tok_io[b] - ptr0), e = min(tok - ptr0, nb - 1);
    for (int j = s0; j <= e && len < max_out - 1; ++j) ob[len++] = body[j];
    if (len < max_out) ob[len++] = fsm.sep_token;
  } else if (!(k8 == 3 && tok != fsm.sep_token)) {
    if (len < max_out) ob[len++] = tok;
  }
  out_len[b] = len;
  tok_io[b] = tok;
  state[b] = ns < 0 ? fsm.done_state : ns;
  if (ns < 0 || ns == fsm.done_state) done[b] = 1;
  else pos[b] = pos[b] + 1;
}

// ---------------------------------------------------------------------------
// copy-constrained decoding (serving/fsm.py COPY_START / COPY_NEXT states): the
// per-row allowed-token mask = the state's schema mask AND the tokens the row may
// copy from its own SMS body.  A value starts at a word boundary of the body (any
// body token not glued to an alphanumeric predecessor; <sep> = an empty value is
// always allowed there); after that the next token must follow the previous one
// somewhere in the body, and <sep> is allowed only where such an occurrence is
// followed by a word boundary (or the end of the body) -- a value never ends
// inside a word split into several tokens.  Boundary: tokens a, b adjacent with
// NOT (a ends alphanumeric AND b starts alphanumeric) (tok_flags, bit 0 = starts,
// bit 1 = ends alphanumeric; byte-level BPE puts a word's leading blank in its
// first token).  One wave per row builds the bit set in LDS (V/32 words), then
// writes the full mask row; rows in non-copy states are skipped (their mask row
// is never read: the consumers check copy_kind[state] first).  A row left with an
// empty set decodes <sep> (the consumers' nothing-allowed fallback).  Consumers:
// the lm_head arg-max epilogue (EPI 4), fsm_sample_kernel, spec_verify_kernel.
// ---------------------------------------------------------------------------
#define COPY_MAX_WORDS 512  // V <= 16384

__global__ void __launch_bounds__(256) copy_mask_kernel(
    FsmTables fsm, const int* __restrict__ copy_kind, const uint8_t* __restrict__ tok_flags,
    const int* __restrict__ row_state, const int* __restrict__ prev_tok, const int* __restrict__ row_slot,
    const int* __restrict__ body_buf, const int* __restrict__ body_len, int LB, int n,
    uint32_t* __restrict__ row_masks) {
  __shared__ uint32_t bits[4][COPY_MAX_WORDS];
  const int wid = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int r = blockIdx.x * 4 + wid;
  if (r >= n) return;  // wave-uniform: no block barrier below
  const int s = row_state[r];
  const int kind = copy_kind[s];
  if (kind == 0) return;
  const int words = fsm.V >> 5;
  uint32_t* b = bits[wid];
  for (int w = lane; w < words; w += 64) b[w] = 0u;
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  const int sl = row_slot[r];
  const int bl = min(body_len[sl], LB);
  const int* body = body_buf + (size_t)sl * LB;
  const int prev = prev_tok[r];
  const int sep = fsm.sep_token;
  auto flags = [&](int t) -> int { return (t >= 0 && t < fsm.V) ? (int)tok_flags[t] : 0; };
  for (int j = lane; j < bl; j += 64) {
    const int t = body[j];
    int cand = -1;
    bool end_ok = false;
    if (kind == 1) {
      const bool glued = j > 0 && (flags(body[j - 1]) & 2) && (flags(t) & 1);
      if (!glued) cand = t;
    } else if (t == prev) {
      const int nx = j + 1 < bl ? body[j + 1] : -1;
      cand = nx;
      end_ok = nx < 0 || !((flags(t) & 2) && (flags(nx) & 1));
    }
    if (cand >= 0 && cand < fsm.V) atomicOr(&b[cand >> 5], 1u << (cand & 31));
    if (end_ok) atomicOr(&b[sep >> 5], 1u << (sep & 31));
  }
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  const uint32_t* m = fsm.masks + (size_t)fsm.state_mask[s] * words;
  const int sw = sep >> 5;
  const uint32_t sbit = kind == 1 ? 1u << (sep & 31) : 0u;  // an empty value: always allowed
  uint32_t* out = row_masks + (size_t)r * words;
  for (int w = lane; w < words; w += 64) out[w] = (b[w] | (w == sw ? sbit : 0u)) & m[w];
}

// ---------------------------------------------------------------------------
// verify: grid = B blocks of 256 threads.
// ---------------------------------------------------------------------------
__global__ void __launch_bounds__(256) spec_verify_kernel(
    const uint16_t* __restrict__ logits, int ldl, const uint32_t* __restrict__ masks, const int* __restrict__ state_mask,
    int* __restrict__ state, const int* __restrict__ next_sep, const int* __restrict__ next_tok,
    const int* __restrict__ enum_tok, const int* __restrict__ enum_next, int E, int sep_token, int done_state,
    int* __restrict__ tok_buf, int* __restrict__ out_buf, int* __restrict__ out_len, int* __restrict__ done,
    int* __restrict__ pos, const int* __restrict__ x_tok, const int* __restrict__ row_start,
    const int* __restrict__ row_nd, int* __restrict__ accepted, int max_out, int V, const int* __restrict__ copy_kind,
    const uint32_t* __restrict__ row_masks) {
  const int b = blockIdx.x;
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  __shared__ float bv[4];
  __shared__ int bi[4];
  __shared__ int s_go, s_state;
  if (done[b]) {  // block-uniform
    if (tid == 0 && accepted != nullptr) accepted[b] = 0;
    return;
  }
  const int st = row_start[b], nd = row_nd[b];
  int s = state[b];
  int emitted = 0;
  for (int i = 0; i <= nd; ++i) {
    // copy state: pseudo-row st + i's own mask (built for x_state[st + i] == s: the
    // drafts before it were accepted, or the loop would have stopped)
    const uint32_t* mrow = (copy_kind != nullptr && copy_kind[s]) ? row_masks + (size_t)(st + i) * (V >> 5)
                                                                   : masks + (size_t)state_mask[s] * (V >> 5);
    const uint16_t* lrow = logits + (size_t)(st + i) * ldl;
    float best = -INFINITY;
    int besti = 0x7fffffff;
    const int nvec = V >> 3;
    for (int c = tid; c < nvec; c += 256) {
      const uint32_t bits = (mrow[c >> 2] >> ((c & 3) * 8)) & 0xffu;
      if (!bits) continue;
      const uint4 raw = *reinterpret_cast<const uint4*>(lrow + 8 * c);
      const uint32_t w[4] = {raw.x, raw.y, raw.z, raw.w};
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        if (bits & (1u << j)) {
          const int idx = 8 * c + j;
          const float v = sp_bf2f((uint16_t)(w[j >> 1] >> ((j & 1) * 16)));
          if (v > best || (v == best && idx < besti)) { best = v; besti = idx; }
        }
      }
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
      const float ov = __shfl_xor(best, o, 64);
      const int oi = __shfl_xor(besti, o, 64);
      if (ov > best || (ov == best && oi < besti)) { best = ov; besti = oi; }
    }
    if (lane == 0) { bv[wid] = best; bi[wid] = besti; }
    __syncthreads();
    if (tid == 0) {
      for (int w = 1; w < 4; ++w)
        if (bv[w] > best || (bv[w] == best && bi[w] < besti)) { best = bv[w]; besti = bi[w]; }
      const int tok = (besti == 0x7fffffff) ? sep_token : besti;
      int ns;
      if (tok == sep_token) {
        ns = next_sep[s];
      } else {
        ns = next_tok[s];
        if (E > 0 && ns == -2) {
          ns = -1;
          for (int e = 0; e < E; ++e)
            if (enum_tok[s * E + e] == tok) { ns = enum_next[s * E + e]; break; }
        }
      }
      const int len = out_len[b];
      out_buf[(size_t)b * max_out + len] = tok;
      out_len[b] = len + 1;
      tok_buf[b] = tok;
      const int nstate = ns < 0 ? done_state : ns;
      state[b] = nstate;
      int go = 0;
      if (ns < 0 || ns == done_state || len + 1 >= max_out) {
        done[b] = 1;
      } else {
        pos[b] = pos[b] + 1;
        go = (i < nd) && (tok == x_tok[st + i + 1]);  // next query token is exactly this one
      }
      s_go = go;
      s_state = nstate;
    }
    __syncthreads();
    ++emitted;
    s = s_state;
    if (!s_go) break;
  }
  if (tid == 0 && accepted != nullptr) accepted[b] = emitted;
}

// ---------------------------------------------------------------------------
// Candidate-sparse lm_head + masked arg-max (copy-constrained decoding).  Under the
// copy constraint a row may only emit <sep> or tokens of its own SMS body (copy
// states), or the few tokens of an enum / forced state: ~2 candidates mid-copy, ~40 at
// a field start, of 8 192.  The dense lm_head GEMM (EPI 4 of gemm_fused_kernel)
// computes all 8 192 logits of every pseudo-row to arg-max over that handful; here one
// wave per row builds the row's allowed set exactly as copy_mask_kernel does (bit set
// in LDS, AND the state's schema mask), compacts it to a candidate list, and dots the
// row's final-normed hidden state with the candidates' (norm-folded) lm_head rows
// only: 16 candidates per pass, four lanes per candidate reading its W row as 16-B
// chunks against the row staged in LDS.
// Each logit is rounded to bf16 like the dense epilogue's staged tile and reduced with
// the same key (larger value, then smaller token id), so best[] feeds fsm_commit /
// spec_verify_keys unchanged.  The row scale rsqrt(mean(x^2) + eps) is computed from
// the row itself.  Rows past n, and the wave's candidate overflow, never occur: the
// host checks that no non-copy state allows more than SPARSE_MAX_CAND tokens and the
// body is at most LB <= SPARSE_MAX_CAND - 1 tokens.
// ---------------------------------------------------------------------------
#define SPARSE_MAX_CAND 256
#define SPARSE_MAX_HL 16  // hidden <= 1024

static __device__ __forceinline__ unsigned long long sp_argmax_key(float v, int idx) {
  const uint32_t b = __float_as_uint(v + 0.0f);
  const uint32_t k = (b & 0x80000000u) ? ~b : (b | 0x80000000u);
  return ((unsigned long long)k << 32) | (unsigned long long)(0xFFFFFFFFu - (uint32_t)idx);
}

__global__ void __launch_bounds__(256) sparse_argmax_kernel(
    FsmTables fsm, const int* __restrict__ copy_kind, const uint8_t* __restrict__ tok_flags,
    const uint16_t* __restrict__ h, int ldh, const uint16_t* __restrict__ W, int H, float eps,
    const int* __restrict__ row_state, const int* __restrict__ prev_tok, const int* __restrict__ row_slot,
    const int* __restrict__ body_buf, const int* __restrict__ body_len, int LB, int n, int ptr0, int n_pos,
    unsigned long long* __restrict__ best) {
  __shared__ uint32_t bits[4][COPY_MAX_WORDS];
  __shared__ int cand[4][SPARSE_MAX_CAND];
  __shared__ int ncand[4];
  __shared__ __attribute__((aligned(16))) uint16_t hbuf[4][8 * SPARSE_MAX_HL * 8];  // the row, bf16
  const int wid = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int r = blockIdx.x * 4 + wid;
  if (r >= n) return;  // wave-uniform: no block barrier below
  const int s = row_state[r];
  const int kind = copy_kind != nullptr ? copy_kind[s] : 0;
  const int words = fsm.V >> 5;
  const uint32_t* m = fsm.masks + (size_t)fsm.state_mask[s] * words;
  uint32_t* b = bits[wid];
  int* cl = cand[wid];
  if (lane == 0) ncand[wid] = 0;
  if (kind != 0) {  // the row's copy set (copy_mask_kernel's rules)
    for (int w = lane; w < words; w += 64) b[w] = 0u;
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    const int sl = row_slot[r];
    const int bl = min(body_len[sl], LB);
    const int* body = body_buf + (size_t)sl * LB;
    const int prev = prev_tok[r];
    const int sep = fsm.sep_token;
    auto flags = [&](int t) -> int { return (t >= 0 && t < fsm.V) ? (int)tok_flags[t] : 0; };
    const int k8 = kind & 0xff, cls = (kind >> 16) & 0xff;
    if (k8 == 3) {
      // span start (serving/fsm.py build_span_fsm): pointer ptr0 + j to a body token at a
      // word boundary and in the field's class; never the closing <ans> (position bl-1);
      // and only a start that HAS an end (the end state has no <sep>, so a
      // start glued into an out-of-class token -- "1500р" -- would end the answer):
      // some e in [j, j + cap) with j..e in class and a word boundary after e
      const int np = min(bl - 1, n_pos);
      const int cap = (kind >> 8) & 0xff;
      const bool no_mask = (cls & (4 | 8)) != 0;  // dates / numbers never start right after a card mask
      for (int j = lane; j < np; j += 64) {
        const int t = body[j];
        const int fp = j > 0 ? flags(body[j - 1]) : 0;
        const bool glued = (fp & 2) && (flags(t) & 1);
        if (!glued && (cls == 0 || (flags(t) & cls)) && !(no_mask && (fp & 64))) {
          bool has_end = cap == 0;  // (an FSM built without caps in its start states)
          const int nb = bl - 1;
          for (int e = j; !has_end && e < min(nb, j + cap); ++e) {
            const int te = body[e];
            if (cls && !(flags(te) & cls)) break;
            const int nx = e + 1 < nb ? body[e + 1] : -1;
            has_end = nx < 0 || !((flags(te) & 2) && (flags(nx) & 1));
          }
          const int c = ptr0 + j;
          if (has_end && c < fsm.V) atomicOr(&b[c >> 5], 1u << (c & 31));
        }
      }
      if (lane == 0) atomicOr(&b[sep >> 5], 1u << (sep & 31));  // an empty value
    } else if (k8 == 4) {
      // span end: lane l is end position e = start + l (caps <= 64); every token from the
      // start to e in the class (the first out-of-class token by one wave ballot), e
      // within the cap and followed by a word boundary
      const int cap = (kind >> 8) & 0xff, nb = bl - 1, s0 = prev - ptr0;
      if (s0 >= 0 && s0 < nb) {  // row-uniform
        const int e = s0 + lane;
        const bool inr = lane < cap && e < nb;
        const int t = inr ? body[e] : 0;
        const bool inc = inr && (cls == 0 || (flags(t) & cls));
        const unsigned long long bad = __ballot(!inc);
        const int first_bad = bad ? __builtin_ctzll(bad) : 64;
        if (inr && lane < first_bad) {
          const int nx = e + 1 < nb ? body[e + 1] : -1;
          const int c = ptr0 + e;
          if ((nx < 0 || !((flags(t) & 2) && (flags(nx) & 1))) && c < fsm.V)
            atomicOr(&b[c >> 5], 1u << (c & 31));
        }
      }
    } else {
      for (int j = lane; j < bl; j += 64) {
        const int t = body[j];
        int c = -1;
        bool end_ok = false;
        if (k8 == 1) {
          const bool glued = j > 0 && (flags(body[j - 1]) & 2) && (flags(t) & 1);
          if (!glued) c = t;
        } else if (t == prev) {
          const int nx = j + 1 < bl ? body[j + 1] : -1;
          c = nx;
          end_ok = nx < 0 || !((flags(t) & 2) && (flags(nx) & 1));
        }
        if (c >= 0 && c < fsm.V) atomicOr(&b[c >> 5], 1u << (c & 31));
        if (end_ok) atomicOr(&b[sep >> 5], 1u << (sep & 31));
      }
      if (k8 == 1 && lane == 0) atomicOr(&b[sep >> 5], 1u << (sep & 31));  // an empty value
    }
  }
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  // compact the allowed set (copy set AND schema mask; a non-copy row: the schema mask)
  for (int w = lane; w < words; w += 64) {
    uint32_t x = m[w];
    if (kind != 0) x &= b[w];
    while (x) {
      const int bit = __builtin_ctz(x);
      x &= x - 1u;
      const int k = atomicAdd(&ncand[wid], 1);
      if (k < SPARSE_MAX_CAND) cl[k] = 32 * w + bit;
    }
  }
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  const int nc = min(ncand[wid], SPARSE_MAX_CAND);
  // the row's hidden state, staged in LDS as bf16 (16-B chunks), and its RMSNorm scale
  const uint16_t* hr = h + (size_t)r * ldh;
  uint16_t* hb = hbuf[wid];
  const int nch = H >> 3;  // 16-B chunks of the row
  float ss = 0.f;
  for (int k = lane; k < nch; k += 64) {
    const uint4 u = *reinterpret_cast<const uint4*>(hr + 8 * k);
    *reinterpret_cast<uint4*>(hb + 8 * k) = u;
    const uint32_t w4[4] = {u.x, u.y, u.z, u.w};
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const float lo = sp_bf2f((uint16_t)(w4[e] & 0xffffu)), hi = sp_bf2f((uint16_t)(w4[e] >> 16));
      ss = fmaf(lo, lo, fmaf(hi, hi, ss));
    }
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) ss += __shfl_xor(ss, o, 64);
  const float rs = rsqrtf(ss / (float)H + eps);
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  // 16 candidates per pass: lane = 4 c + q dots candidate c over the q-th quarter of the
  // dims (16-B W chunks; the h chunk is an LDS broadcast to the 16 lanes of quarter q),
  // then the 4 quarters are summed with two shuffles
  const int c = lane >> 2, q = lane & 3, QD = H >> 2, qch = QD >> 3;
  unsigned long long bk = 0ull;
  for (int c0 = 0; c0 < nc; c0 += 16) {
    const int tk = c0 + c < nc ? cl[c0 + c] : -1;
    float part = 0.f;
    if (tk >= 0) {
      const uint16_t* wr = W + (size_t)tk * H + q * QD;
      const uint16_t* hq = hb + q * QD;
      for (int k = 0; k < qch; ++k) {
        const uint4 wu = *reinterpret_cast<const uint4*>(wr + 8 * k);
        const uint4 hu = *reinterpret_cast<const uint4*>(hq + 8 * k);
        const uint32_t a4[4] = {wu.x, wu.y, wu.z, wu.w}, b4[4] = {hu.x, hu.y, hu.z, hu.w};
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          part = fmaf(sp_bf2f((uint16_t)(a4[e] & 0xffffu)), sp_bf2f((uint16_t)(b4[e] & 0xffffu)), part);
          part = fmaf(sp_bf2f((uint16_t)(a4[e] >> 16)), sp_bf2f((uint16_t)(b4[e] >> 16)), part);
        }
      }
    }
    part += __shfl_xor(part, 1, 64);
    part += __shfl_xor(part, 2, 64);
    if (tk >= 0 && q == 0) {
      const __bf16 lb = (__bf16)(part * rs);  // the dense epilogue's staged bf16 logit
      const unsigned long long k2 = sp_argmax_key(sp_bf2f(__builtin_bit_cast(uint16_t, lb)), tk);
      bk = k2 > bk ? k2 : bk;
    }
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    const unsigned long long ok = __shfl_xor(bk, o, 64);
    bk = ok > bk ? ok : bk;
  }
  if (lane == 0) best[r] = bk;
}

extern "C" {

static FsmTables make_fsm(const void* masks, const int* state_mask, const int* next_sep, const int* next_tok,
                          const int* enum_tok, const int* enum_next, int E, int sep_token, int done_state, int V) {
  return FsmTables{(const uint32_t*)masks, state_mask, next_sep, next_tok, enum_tok, enum_next, E, sep_token,
                   done_state, V};
}

int sg_spec_plan(const void* masks, const int* state_mask, const int* next_sep, const int* next_tok,
                 const int* enum_tok, const int* enum_next, int E, int done_state, int V, const int* state,
                 int* x_state, int B, int K, int T_cap, int sep_token, int scratch_slot, const int* tok_buf, const int* pos,
                 const int* slot, const int* done, const int* out_buf, const int* out_len, int max_out,
                 const int* body_buf, const int* body_len, int LB, const void* delim, const int* forced, int policy,
                 int* draft_buf, int* x_tok, int* x_pos, int* x_slot, int* x_done, int* row_start, int* row_nd,
                 int* meta, hipStream_t stream) {
  if (K < 0 || K > SPEC_MAX_K || T_cap < B || B <= 0 || policy < 0 || policy > 1) return -1;
  const FsmTables f = make_fsm(masks, state_mask, next_sep, next_tok, enum_tok, enum_next, E, sep_token, done_state, V);
  const int grid = (B + 255) / 256;
  hipLaunchKernelGGL(spec_draft_kernel, dim3(grid), dim3(256), 0, stream, f, state, B, K, sep_token, tok_buf, slot, done,
                     out_buf, out_len, max_out, body_buf, body_len, LB, (const uint8_t*)delim, forced, policy, draft_buf,
                     row_nd);
  hipLaunchKernelGGL(spec_scan_kernel, dim3(1), dim3(SPEC_THREADS), 0, stream, B, K, T_cap, row_start, row_nd, meta);
  hipLaunchKernelGGL(spec_fill_kernel, dim3(grid), dim3(256), 0, stream, f, state, B, T_cap, scratch_slot, tok_buf, pos,
                     slot, done, draft_buf, row_start, row_nd, meta, x_tok, x_pos, x_slot, x_done, x_state);
  return (int)hipGetLastError();
}

int sg_spec_verify(const void* logits, int ldl, const void* masks, const int* state_mask, int* state,
                   const int* next_sep, const int* next_tok, const int* enum_tok, const int* enum_next, int E,
                   int sep_token, int done_state, int* tok_buf, int* out_buf, int* out_len, int* done, int* pos,
                   const int* x_tok, const int* row_start, const int* row_nd, int* accepted, int max_out, int V, int B,
                   const int* copy_kind, const void* row_masks, hipStream_t stream) {
  if (V % 32 || ldl % 8 || (copy_kind != nullptr && row_masks == nullptr)) return -1;
  if (B == 0) return 0;
  hipLaunchKernelGGL(spec_verify_kernel, dim3(B), dim3(256), 0, stream, (const uint16_t*)logits, ldl,
                     (const uint32_t*)masks, state_mask, state, next_sep, next_tok, enum_tok, enum_next, E, sep_token,
                     done_state, tok_buf, out_buf, out_len, done, pos, x_tok, row_start, row_nd, accepted, max_out, V,
                     copy_kind, (const uint32_t*)row_masks);
  return (int)hipGetLastError();
}

int sg_spec_verify_keys(const void* best, const void* masks, const int* state_mask, const int* next_sep,
                        const int* next_tok, const int* enum_tok, const int* enum_next, int E, int sep_token,
                        int done_state, int V, int* state, int* tok_buf, int* out_buf, int* out_len, int* done, int* pos,
                        const int* x_tok, const int* row_start, const int* row_nd, int* accepted, int max_out, int B,
                        void* counts, hipStream_t stream) {
  if (B == 0) return 0;
  const FsmTables f = make_fsm(masks, state_mask, next_sep, next_tok, enum_tok, enum_next, E, sep_token, done_state, V);
  hipLaunchKernelGGL(spec_verify_keys_kernel, dim3((B + 255) / 256), dim3(256), 0, stream, f,
                     (const unsigned long long*)best, state, tok_buf, out_buf, out_len, done, pos, x_tok, row_start,
                     row_nd, accepted, max_out, B, (unsigned long long*)counts);
  return (int)hipGetLastError();
}

int sg_fsm_commit(const void* best, const int* row_map, const void* masks, const int* state_mask,
                  const int* next_sep, const int* next_tok, const int* enum_tok, const int* enum_next, int E,
                  int sep_token, int done_state, int V, int* state, int* tok_io, int* out_buf, int* out_len, int* done,
                  int* pos,
                  int max_out, int B, hipStream_t stream) {
  if (B == 0) return 0;
  const FsmTables f = make_fsm(masks, state_mask, next_sep, next_tok, enum_tok, enum_next, E, sep_token, done_state, V);
  hipLaunchKernelGGL(fsm_commit_kernel, dim3((B + 255) / 256), dim3(256), 0, stream, f,
                     (const unsigned long long*)best, row_map, state, tok_io, out_buf, out_len, done, pos, max_out, B);
  return (int)hipGetLastError();
}

// candidate-sparse lm_head + masked arg-max for n rows (sparse_argmax_kernel): best[r]
// = the arg-max key over the tokens row r may emit (its state's schema mask, AND its copy
// set in a copy state).  h [n][ldh] bf16 un-normed, W [V][H] bf16 with the final norm
// folded in.
int sg_sparse_argmax(const void* masks, const int* state_mask, int sep_token, int V, const int* copy_kind,
                     const void* tok_flags, const void* h, int ldh, const void* W, int H, float eps,
                     const int* row_state, const int* prev_tok, const int* row_slot, const int* body_buf,
                     const int* body_len, int LB, int n, int ptr0, int n_pos, void* best, hipStream_t stream) {
  if (V % 32 || V / 32 > COPY_MAX_WORDS || LB <= 0 || LB >= SPARSE_MAX_CAND || sep_token < 0 || sep_token >= V ||
      H % 64 || H / 64 > SPARSE_MAX_HL || ldh % 8 || (copy_kind && !tok_flags) ||
      (n_pos > 0 && (ptr0 < 0 || ptr0 + n_pos > V || n_pos >= SPARSE_MAX_CAND)))
    return -1;
  if (n == 0) return 0;
  const FsmTables f = make_fsm(masks, state_mask, nullptr, nullptr, nullptr, nullptr, 0, sep_token, 0, V);
  hipLaunchKernelGGL(sparse_argmax_kernel, dim3((n + 3) / 4), dim3(256), 0, stream, f, copy_kind,
                     (const uint8_t*)tok_flags, (const uint16_t*)h, ldh, (const uint16_t*)W, H, eps, row_state,
                     prev_tok, row_slot, body_buf, body_len, LB, n, ptr0, n_pos, (unsigned long long*)best);
  return (int)hipGetLastError();
}

// span-pointer commit (span_commit_kernel) for B key rows.
int sg_span_commit(const void* best, const int* row_map, const void* masks, const int* state_mask,
                   const int* next_sep, const int* next_tok, const int* enum_tok, const int* enum_next, int E,
                   int sep_token, int done_state, int V, const int* copy_kind, const int* row_slot,
                   const int* body_buf, const int* body_len, int LB, int ptr0, int* state, int* tok_io, int* out_buf,
                   int* out_len, int* done, int* pos, int max_out, int B, hipStream_t stream) {
  if (B == 0) return 0;
  if (!copy_kind || !row_slot || !body_buf || !body_len || LB <= 0 || ptr0 < 0 || max_out <= 0) return -1;
  const FsmTables f = make_fsm(masks, state_mask, next_sep, next_tok, enum_tok, enum_next, E, sep_token, done_state, V);
  hipLaunchKernelGGL(span_commit_kernel, dim3((B + 255) / 256), dim3(256), 0, stream, f, copy_kind,
                     (const unsigned long long*)best, row_map, row_slot, body_buf, body_len, LB, ptr0, state, tok_io,
                     out_buf, out_len, done, pos, max_out, B);
  return (int)hipGetLastError();
}

// per-row copy masks (copy_mask_kernel) for n rows: row r in state row_state[r], its
// last emitted token prev_tok[r], its prompt ids body_buf[row_slot[r]]; row_masks
// [n][V/32].  Rows whose state is not a copy state are left untouched.
int sg_copy_masks(const void* masks, const int* state_mask, int sep_token, int V, const int* copy_kind,
                  const void* tok_flags, const int* row_state, const int* prev_tok, const int* row_slot,
                  const int* body_buf, const int* body_len, int LB, int n, void* row_masks, hipStream_t stream) {
  if (V % 32 || V / 32 > COPY_MAX_WORDS || LB <= 0 || sep_token < 0 || sep_token >= V || !tok_flags) return -1;
  if (n == 0) return 0;
  const FsmTables f = make_fsm(masks, state_mask, nullptr, nullptr, nullptr, nullptr, 0, sep_token, 0, V);
  hipLaunchKernelGGL(copy_mask_kernel, dim3((n + 3) / 4), dim3(256), 0, stream, f, copy_kind,
                     (const uint8_t*)tok_flags, row_state, prev_tok, row_slot, body_buf, body_len, LB, n,
                     (uint32_t*)row_masks);
  return (int)hipGetLastError();
}

}  // extern "C"
