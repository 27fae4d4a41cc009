// smsgate_amd — one-forward span extraction head (serving/qa.py, gfx950).
//
// After the prefill forward of `body <ans> q_0 .. q_{nq-1}` (the native prefill,
// csrc/runtime.hip), the last nq rows of every sequence are its query rows.  One
// block per message:
//
//   1. stage the nq query rows (bf16, LDS) and their RMSNorm scales (the final norm's
//      weight is folded into W, ops.fold_norm) and the message's prompt ids / token
//      flags;
//   2. scores: every W row the message needs is read ONCE and dotted with every query
//      row that uses it -- start-pointer row j with the nf start rows, end-pointer row j
//      with the nf end rows, the null row with the start rows, class row c with query
//      row 0.  Four lanes per W row (a quarter of H each, 16-B chunks), 16 W rows per
//      wave pass, fp32 accumulation, fp32 scores in LDS;
//   3. decode (one wave per field, fields w and w + 4): the class is the arg-max of the
//      four class scores; per copied field the null decision (null score >= every
//      valid start's score, or no valid pair) and the joint arg-max of
//      start[s] + end[e] over valid pairs -- s at a word boundary and in the field's
//      class (and, for dates / numbers, not right after a card mask), e >= s within
//      the cap, every token s..e in class and none a line break, the first / last
//      token with the field kind's edge flags (s_need / e_need: a number starts and
//      ends with a digit ...), e followed by a word boundary.  Word boundary: NOT (a
//      ends with a letter and b starts with one, or a ends with a digit and b starts
//      with one), and a lone separator between a digit and a three-digit group joins
//      them ("218" "," "993").  A date span with no time of day then takes the time
//      token right before (else right after) it when that longer span is valid, and a
//      span ending in a digit a following AM / PM.
//      One lane per start, its ends scanned in order;
//      ties go to the lower start, then the lower end (serving/qa.py qa_decode_ref);
//      Confidence: the probability of each decision under the distributions the head
//      is trained on (serving/qa.py qa_loss) -- the class softmax, per field the start
//      softmax over the body positions and null, and the end softmax over the body
//      positions -- a field's confidence the product of its start and end probabilities
//      (its null probability when null), the answer's the least of them.  A transaction
//      answer under p.min_conf is turned into p.abstain_cls (serving/qa.py qa_decode_ref);
//   4. the answer in the copy format (class tokens, <sep>, each field's body tokens
//      and <sep>; a rejection class: only its tokens and <sep>) into out_buf.
//
// Optional outputs for tests: the raw scores and the decoded (class, spans).
#include <hip/hip_runtime.h>
#include <stdint.h>

#define QA_MAX_NF 8
#define QA_MAX_NQ 24
#define QA_MAX_POS 160
#define QA_NCLS 4
#define QA_MAX_CLS_TOK 8

#define QF_SL 1
#define QF_SD 2
#define QF_EL 4
#define QF_ED 8
#define QF_MASK 16
#define QF_NO_START_AFTER_MASK (32 | 64)  // date | number class bits
#define QF_NL 512      // contains a line break
#define QF_LD 8192     // last char a digit
#define QF_GRP3 16384  // exactly three ASCII digits
#define QF_SEP 32768   // a lone "," "." "'"
#define QF_TIME 65536  // a whole time of day (" 22:09")
#define QF_AMPM (1 << 18)  // " AM" / " PM"
#define QF_AP (1 << 19)    // " A" / " P" (a split " AM" / " PM")
#define QF_M (1 << 20)     // "M"
#define QF_CARDL (1 << 22)  // " CARD" (normalize_body's "CARD:7538")
#define QF_COLON (1 << 23)  // a lone ":"
#define QF_XMASK (1 << 24)  // x / X letters only ("XXXX" of "XXXX1438")

struct QAParams {
  int nf, nq, n_pos;
  int start_row[QA_MAX_NF];
  int end_row[QA_MAX_NF];
  int cls_bits[QA_MAX_NF];
  int cap[QA_MAX_NF];
  int off_end, off_null, off_cls;  // W rows relative to start-pointer row 0
  int cls_tok[QA_NCLS][QA_MAX_CLS_TOK];
  int cls_len[QA_NCLS];
  int reject_mask;  // bit c: class c is a non-transaction (no fields)
  int sep, max_out;
  int s_need[QA_MAX_NF];  // edge flags the first token must all have (serving/qa.py EDGE_RULES)
  int e_need[QA_MAX_NF];  // ... and the last token
  int absorb[QA_MAX_NF];  // 1: a span without a time of day takes an adjacent one (dates)
  // abstention: a transaction answer whose confidence (the least probable of its
  // decisions, below) is under min_conf becomes class abstain_cls (a non-transaction:
  // null fields -> the unmatched DLQ) instead of being published with a doubtful field
  float min_conf;
  int abstain_cls;
};

static __device__ __forceinline__ float qa_bf2f(uint16_t v) { return __uint_as_float(((uint32_t)v) << 16); }

static __device__ __forceinline__ bool qa_glued(uint32_t fa, uint32_t fb) {
  return ((fa & QF_EL) && (fb & QF_SL)) || ((fa & QF_ED) && (fb & QF_SD));
}

// s may start a value of class bits `cls` with first-token edge flags `sneed`
static __device__ __forceinline__ bool qa_start_ok(const uint32_t* fb, int s, int cls, int sneed) {
  const uint32_t fs = fb[s];
  bool ok = ((cls == 0) || (fs & cls)) && !(fs & QF_NL) && (fs & sneed) == (uint32_t)sneed;
  if (ok && s > 0) {
    const uint32_t fp = fb[s - 1];
    ok = !qa_glued(fp, fs) && !((cls & QF_NO_START_AFTER_MASK) && (fp & QF_MASK)) &&
         !((cls & QF_NO_START_AFTER_MASK) && (((fp & QF_XMASK) && (fs & QF_SD)) ||
                                             (s > 1 && (fp & QF_COLON) && (fb[s - 2] & QF_CARDL)))) &&
         !(s > 1 && (fp & QF_SEP) && (fs & QF_GRP3) && (fb[s - 2] & QF_LD));
  }
  return ok;
}

// e may end a value (its own token already known in class): last-token edge flags and a
// word boundary after it
static __device__ __forceinline__ bool qa_end_ok(const uint32_t* fb, int n, int e, int eneed) {
  const uint32_t fe = fb[e];
  if ((fe & eneed) != (uint32_t)eneed) return false;
  if (e + 1 < n) {
    const uint32_t fn = fb[e + 1];
    if (qa_glued(fe, fn)) return false;
    if ((fe & QF_SEP) && (fn & QF_GRP3) && e > 0 && (fb[e - 1] & QF_LD)) return false;
    if ((fe & QF_LD) && (fn & QF_SEP) && e + 2 < n && (fb[e + 2] & QF_GRP3)) return false;
  }
  return true;
}

static __device__ __forceinline__ bool qa_in_cls(uint32_t f, int cls) {
  return ((cls == 0) || (f & cls)) && !(f & QF_NL);
}

__global__ void __launch_bounds__(256) qa_decode_kernel(
    QAParams p, const uint16_t* __restrict__ h, int ldh, const uint16_t* __restrict__ W, int H, float eps,
    const int* __restrict__ cu, const int* __restrict__ ids, const uint32_t* __restrict__ flags, int V,
    int* __restrict__ out_buf, int* __restrict__ out_len, float* __restrict__ dbg_scores,
    int* __restrict__ dbg_spans, float* __restrict__ out_conf, int compact) {
  extern __shared__ __attribute__((aligned(16))) uint16_t hq[];  // [nq][H] bf16
  __shared__ float rs[QA_MAX_NQ];
  __shared__ float sc_start[QA_MAX_NF][QA_MAX_POS];
  __shared__ float sc_end[QA_MAX_NF][QA_MAX_POS];
  __shared__ float sc_null[QA_MAX_NF];
  __shared__ float sc_cls[QA_NCLS];
  __shared__ uint32_t fb[QA_MAX_POS];
  __shared__ int body[QA_MAX_POS];
  __shared__ int span_s[QA_MAX_NF], span_e[QA_MAX_NF];
  __shared__ float conf_f[QA_MAX_NF];
  __shared__ int cls_sel;

  const int m = blockIdx.x;
  const int tid = threadIdx.x, wid = tid >> 6, lane = tid & 63;
  const int nq = p.nq, nf = p.nf;
  const int r0 = cu[m], r1 = cu[m + 1];
  // query rows: the last nq rows of the sequence, or (compact: the engine ran the last
  // layer on the query rows only) rows m * nq .. of a query-rows-only h
  const int qrow0 = compact ? m * nq : r1 - nq;
  // pointable positions (the body; <ans> excluded); >= 0 even for a malformed sequence
  // (the host refuses empty prompts, serving/qa_engine.py), so the class rows are scored
  const int n = max(0, min(r1 - nq - r0 - 1, p.n_pos));
  const int nch = H >> 3;                       // 16-B chunks per row

  // ---- 1. stage
  for (int k = tid; k < nq * nch; k += 256) {
    const int q = k / nch, c = k - q * nch;
    *reinterpret_cast<uint4*>(hq + (size_t)q * H + 8 * c) =
        *reinterpret_cast<const uint4*>(h + (size_t)(qrow0 + q) * ldh + 8 * c);
  }
  for (int j = tid; j < n; j += 256) {
    const int t = ids[r0 + j];
    body[j] = t;
    fb[j] = (t >= 0 && t < V) ? flags[t] : 0u;
  }
  __syncthreads();
  for (int q = wid; q < nq; q += 4) {
    float ss = 0.f;
    const uint32_t* hr = reinterpret_cast<const uint32_t*>(hq + (size_t)q * H);
    for (int k = lane; k < (H >> 1); k += 64) {
      const uint32_t u = hr[k];
      const float lo = qa_bf2f((uint16_t)(u & 0xffffu)), hi = qa_bf2f((uint16_t)(u >> 16));
      ss = fmaf(lo, lo, fmaf(hi, hi, ss));
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) ss += __shfl_xor(ss, o, 64);
    if (lane == 0) rs[q] = rsqrtf(ss / (float)H + eps);
  }
  __syncthreads();

  // ---- 2. scores.  Items: [0, n) start rows, [n, 2n) end rows, 2n the null row,
  // 2n+1 .. 2n+4 the class rows.  16 items per wave pass, four lanes each.
  const int items = 2 * n + 1 + QA_NCLS;
  const int ci = lane >> 2, qd = lane & 3, QD = H >> 2, qch = QD >> 3;
  for (int i0 = wid * 16; i0 < items; i0 += 64) {
    const int it = i0 + ci;
    float acc[QA_MAX_NF];
#pragma unroll
    for (int f = 0; f < QA_MAX_NF; ++f) acc[f] = 0.f;
    int wrow = -1, kind = 0;  // kind 0 start, 1 end, 2 null, 3 class
    if (it < n) { wrow = it; kind = 0; }
    else if (it < 2 * n) { wrow = p.off_end + (it - n); kind = 1; }
    else if (it == 2 * n) { wrow = p.off_null; kind = 2; }
    else if (it < items) { wrow = p.off_cls + (it - 2 * n - 1); kind = 3; }
    if (wrow >= 0) {
      const uint16_t* wr = W + (size_t)wrow * H + qd * QD;
      for (int k = 0; k < qch; ++k) {
        const uint4 wu = *reinterpret_cast<const uint4*>(wr + 8 * k);
        const uint32_t a4[4] = {wu.x, wu.y, wu.z, wu.w};
        float wf[8];
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          wf[2 * e] = qa_bf2f((uint16_t)(a4[e] & 0xffffu));
          wf[2 * e + 1] = qa_bf2f((uint16_t)(a4[e] >> 16));
        }
        if (kind == 3) {
          const uint4 hu = *reinterpret_cast<const uint4*>(hq + qd * QD + 8 * k);  // query row 0
          const uint32_t b4[4] = {hu.x, hu.y, hu.z, hu.w};
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            acc[0] = fmaf(wf[2 * e], qa_bf2f((uint16_t)(b4[e] & 0xffffu)), acc[0]);
            acc[0] = fmaf(wf[2 * e + 1], qa_bf2f((uint16_t)(b4[e] >> 16)), acc[0]);
          }
        } else {
#pragma unroll
          for (int f = 0; f < QA_MAX_NF; ++f) {
            if (f < nf) {
              const int q = kind == 1 ? p.end_row[f] : p.start_row[f];
              const uint4 hu = *reinterpret_cast<const uint4*>(hq + (size_t)q * H + qd * QD + 8 * k);
              const uint32_t b4[4] = {hu.x, hu.y, hu.z, hu.w};
#pragma unroll
              for (int e = 0; e < 4; ++e) {
                acc[f] = fmaf(wf[2 * e], qa_bf2f((uint16_t)(b4[e] & 0xffffu)), acc[f]);
                acc[f] = fmaf(wf[2 * e + 1], qa_bf2f((uint16_t)(b4[e] >> 16)), acc[f]);
              }
            }
          }
        }
      }
    }
#pragma unroll
    for (int f = 0; f < QA_MAX_NF; ++f) {
      acc[f] += __shfl_xor(acc[f], 1, 64);
      acc[f] += __shfl_xor(acc[f], 2, 64);
    }
    if (wrow >= 0 && qd == 0) {
      if (kind == 3) {
        sc_cls[it - 2 * n - 1] = acc[0] * rs[0];
      } else {
#pragma unroll
        for (int f = 0; f < QA_MAX_NF; ++f) {
          if (f < nf) {
            if (kind == 0) sc_start[f][it] = acc[f] * rs[p.start_row[f]];
            else if (kind == 1) sc_end[f][it - n] = acc[f] * rs[p.end_row[f]];
            else sc_null[f] = acc[f] * rs[p.start_row[f]];
          }
        }
      }
    }
  }
  __syncthreads();

  // ---- 3. decode
  if (tid == 0) {
    int c = 0;
    for (int k = 1; k < QA_NCLS; ++k)
      if (sc_cls[k] > sc_cls[c]) c = k;
    cls_sel = c;
  }
  for (int f = wid; f < nf; f += 4) {
    const int cls = p.cls_bits[f], cap = p.cap[f], sneed = p.s_need[f], eneed = p.e_need[f];
    float top = -INFINITY;  // best valid start score
    float best = -INFINITY;
    int bs = 0x7fffffff, be = -1;
    for (int s = lane; s < n; s += 64) {
      if (!qa_start_ok(fb, s, cls, sneed)) continue;
      const float ss = sc_start[f][s];
      top = fmaxf(top, ss);
      const int emax = min(n, s + cap);
      for (int e = s; e < emax; ++e) {
        if (!qa_in_cls(fb[e], cls)) break;
        if (!qa_end_ok(fb, n, e, eneed)) continue;
        const float v = ss + sc_end[f][e];
        if (v > best) { best = v; bs = s; be = e; }  // strict: the lowest end of this start
      }
    }
    // wave: max score, then the lowest start among the lanes that reach it (a lane's
    // starts ascend with its pass, so its first reaching start is its lowest)
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
      top = fmaxf(top, __shfl_xor(top, o, 64));
      const float ob = __shfl_xor(best, o, 64);
      const int os = __shfl_xor(bs, o, 64), oe = __shfl_xor(be, o, 64);
      if (ob > best || (ob == best && os < bs)) { best = ob; bs = os; be = oe; }
    }
    // the field's start (body positions + null) and end (body positions) softmax
    float mxs = -INFINITY, mxe = -INFINITY;
    for (int j = lane; j < n; j += 64) {
      mxs = fmaxf(mxs, sc_start[f][j]);
      mxe = fmaxf(mxe, sc_end[f][j]);
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
      mxs = fmaxf(mxs, __shfl_xor(mxs, o, 64));
      mxe = fmaxf(mxe, __shfl_xor(mxe, o, 64));
    }
    mxs = fmaxf(mxs, sc_null[f]);
    float zs = 0.f, ze = 0.f;
    for (int j = lane; j < n; j += 64) {
      zs += expf(sc_start[f][j] - mxs);
      ze += expf(sc_end[f][j] - mxe);
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
      zs += __shfl_xor(zs, o, 64);
      ze += __shfl_xor(ze, o, 64);
    }
    zs += expf(sc_null[f] - mxs);
    if (lane == 0) {
      const bool null = be < 0 || !(top > sc_null[f]);
      conf_f[f] = null ? expf(sc_null[f] - mxs) / zs
                       : (expf(sc_start[f][bs] - mxs) / zs) * (expf(sc_end[f][be] - mxe) / ze);
      if (!null && p.absorb[f]) {
        bool timed = false;
        for (int j = bs; j <= be; ++j) timed |= (fb[j] & QF_TIME) != 0;
        // the longer span must be a valid pair: start / end rules, in class, within the cap
        if (!timed && bs > 0 && (fb[bs - 1] & QF_TIME) && be - bs + 1 < cap && qa_in_cls(fb[bs - 1], cls) &&
            qa_start_ok(fb, bs - 1, cls, sneed))
          bs -= 1;
        else if (!timed && be + 1 < n && (fb[be + 1] & QF_TIME) && be - bs + 1 < cap && qa_in_cls(fb[be + 1], cls) &&
                 qa_end_ok(fb, n, be + 1, eneed))
          be += 1;
        // then a span ending in a digit takes a following AM / PM
        if (fb[be] & QF_LD) {
          if (be + 1 < n && (fb[be + 1] & QF_AMPM) && be - bs + 1 < cap && qa_in_cls(fb[be + 1], cls) &&
              qa_end_ok(fb, n, be + 1, eneed))
            be += 1;
          else if (be + 2 < n && (fb[be + 1] & QF_AP) && (fb[be + 2] & QF_M) && be - bs + 2 < cap &&
                   qa_in_cls(fb[be + 1], cls) && qa_in_cls(fb[be + 2], cls) && qa_end_ok(fb, n, be + 2, eneed))
            be += 2;
        }
      }
      span_s[f] = null ? -1 : bs;
      span_e[f] = null ? -1 : be;
    }
  }
  __syncthreads();

  // ---- confidence and abstention
  if (tid == 0) {
    const int c0 = cls_sel;
    float z = 0.f;
    for (int k = 0; k < QA_NCLS; ++k) z += expf(sc_cls[k] - sc_cls[c0]);
    float conf = 1.f / z;
    const bool rej0 = (p.reject_mask >> c0) & 1;
    if (!rej0)
      for (int f = 0; f < nf; ++f) conf = fminf(conf, conf_f[f]);
    if (out_conf != nullptr) out_conf[m] = conf;
    if (!rej0 && conf < p.min_conf) cls_sel = p.abstain_cls;
  }
  __syncthreads();

  // ---- 4. outputs (thread 0 lays out, the block copies)
  __shared__ int off[QA_MAX_NF + 1];
  const int c = cls_sel;
  const bool reject = (p.reject_mask >> c) & 1;
  if (tid == 0) {
    int o = p.cls_len[c] + 1;
    for (int f = 0; f < nf; ++f) {
      off[f] = o;
      if (!reject) o += (span_s[f] >= 0 ? span_e[f] - span_s[f] + 1 : 0) + 1;
    }
    off[nf] = o;
    out_len[m] = min(o, p.max_out);
  }
  __syncthreads();
  int* ob = out_buf + (size_t)m * p.max_out;
  if (tid < p.cls_len[c]) ob[tid] = p.cls_tok[c][tid];
  if (tid == 0) ob[p.cls_len[c]] = p.sep;
  if (!reject) {
    for (int f = 0; f < nf; ++f) {
      const int len = span_s[f] >= 0 ? span_e[f] - span_s[f] + 1 : 0;
      for (int j = tid; j <= len; j += 256) {
        const int o = off[f] + j;
        if (o < p.max_out) ob[o] = j < len ? body[span_s[f] + j] : p.sep;
      }
    }
  }
  if (dbg_spans != nullptr && tid <= 2 * nf) {
    int v = c;
    if (tid > 0) {
      const int f = (tid - 1) >> 1;
      v = reject ? -1 : ((tid - 1) & 1 ? span_e[f] : span_s[f]);
    }
    dbg_spans[(size_t)m * (1 + 2 * nf) + tid] = v;
  }
  if (dbg_scores != nullptr) {
    // [4 class][nf][start n_pos][null][end n_pos] (positions past n: -inf)
    const int per = QA_NCLS + nf * (2 * p.n_pos + 1);
    float* d = dbg_scores + (size_t)m * per;
    for (int k = tid; k < per; k += 256) {
      float v;
      if (k < QA_NCLS) {
        v = sc_cls[k];
      } else {
        const int r = k - QA_NCLS, f = r / (2 * p.n_pos + 1), j = r % (2 * p.n_pos + 1);
        if (j < p.n_pos) v = j < n ? sc_start[f][j] : -INFINITY;
        else if (j == p.n_pos) v = sc_null[f];
        else v = (j - p.n_pos - 1) < n ? sc_end[f][j - p.n_pos - 1] : -INFINITY;
      }
      d[k] = v;
    }
  }
}

// out[t] = table[ids[t]] + (add[t] >= 0 ? table[add[t]] : 0), rounded to bf16 like
// torch's bf16 add (fp32 sum, round to nearest even).  The qa format's prompt rows: a
// message token carries its pointer row, a query token does not.
__global__ void __launch_bounds__(256) embed_rows_add_ids_kernel(const int* __restrict__ ids,
                                                                 const int* __restrict__ add,
                                                                 const uint16_t* __restrict__ table,
                                                                 uint16_t* __restrict__ out, int T, int H, int V) {
  const int nch = H >> 3;
  const long total = (long)T * nch;
  for (long k = (long)blockIdx.x * blockDim.x + threadIdx.x; k < total; k += (long)gridDim.x * blockDim.x) {
    const int t = (int)(k / nch), c = (int)(k - (long)t * nch);
    const int a = ids[t], b = add[t];
    uint4 u = make_uint4(0u, 0u, 0u, 0u);
    if (a >= 0 && a < V) u = *reinterpret_cast<const uint4*>(table + (size_t)a * H + 8 * c);
    if (b >= 0 && b < V) {
      const uint4 v = *reinterpret_cast<const uint4*>(table + (size_t)b * H + 8 * c);
      uint32_t x[4] = {u.x, u.y, u.z, u.w};
      const uint32_t y[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        uint32_t r = 0;
#pragma unroll
        for (int half = 0; half < 2; ++half) {
          const float s = qa_bf2f((uint16_t)(x[e] >> (16 * half))) + qa_bf2f((uint16_t)(y[e] >> (16 * half)));
          uint32_t bits = __float_as_uint(s);
          bits += 0x7fffu + ((bits >> 16) & 1u);  // round to nearest even (no NaN inputs)
          r |= (bits >> 16) << (16 * half);
        }
        x[e] = r;
      }
      u = make_uint4(x[0], x[1], x[2], x[3]);
    }
    *reinterpret_cast<uint4*>(out + (size_t)t * H + 8 * c) = u;
  }
}

extern "C" {

int sg_qa_decode(const void* params, const void* h, int ldh, const void* W, int H, float eps, const int* cu,
                 const int* ids, const void* flags, int V, int* out_buf, int* out_len, void* dbg_scores,
                 void* dbg_spans, void* out_conf, int M, int compact, hipStream_t stream) {
  const QAParams& p = *reinterpret_cast<const QAParams*>(params);
  if (H % 64 || H > 1024 || ldh % 8 || p.nf <= 0 || p.nf > QA_MAX_NF || p.nq <= 0 || p.nq > QA_MAX_NQ ||
      p.n_pos <= 0 || p.n_pos > QA_MAX_POS || p.max_out <= 0 || p.abstain_cls < 0 || p.abstain_cls >= QA_NCLS ||
      !((p.reject_mask >> p.abstain_cls) & 1))
    return -1;
  for (int c = 0; c < QA_NCLS; ++c)
    if (p.cls_len[c] <= 0 || p.cls_len[c] > QA_MAX_CLS_TOK) return -1;
  if (M == 0) return 0;
  const size_t lds = (size_t)p.nq * H * sizeof(uint16_t);
  hipLaunchKernelGGL(qa_decode_kernel, dim3(M), dim3(256), lds, stream, p, (const uint16_t*)h, ldh,
                     (const uint16_t*)W, H, eps, cu, ids, (const uint32_t*)flags, V, out_buf, out_len,
                     (float*)dbg_scores, (int*)dbg_spans, (float*)out_conf, compact);
  return (int)hipGetLastError();
}

int sg_qa_params_size() { return (int)sizeof(QAParams); }

int sg_embed_rows_add_ids(const int* ids, const int* add, const void* table, void* out, int T, int H, int V,
                          hipStream_t stream) {
  if (H % 8) return -1;
  if (T == 0) return 0;
  const long total = (long)T * (H >> 3);
  const int grid = (int)((total + 255) / 256 < 65536 ? (total + 255) / 256 : 65536);
  hipLaunchKernelGGL(embed_rows_add_ids_kernel, dim3(grid), dim3(256), 0, stream, ids, add,
                     (const uint16_t*)table, (uint16_t*)out, T, H, V);
  return (int)hipGetLastError();
}

}  // extern "C"
