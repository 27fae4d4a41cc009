"""One-forward span extraction (the "qa" answer format, VERDICT r04 next #2a).

The span-pointer format (serving/fsm.py build_span_fsm) still decodes
autoregressively: txn_type, then a start and an end pointer per copied field --
~17 sequential decode steps per message, each re-reading the row's keys.  Round 4's
kernel statistics put that decode at 54 % of the GPU time at ~19 rows per message,
against 41 % for the ~41 prefill rows.

This format asks the whole question in ONE forward.  After ``body <ans>`` the
engine appends ``n_queries`` query tokens (ids ``q0 + k``) at the next positions;
the causal model lets every query row attend to the whole body:

* query row 0 classifies the message: its hidden state against the four class
  rows ``cls0 + c`` (TXN_TYPES order: debit, credit, otp, unknown).  ``otp`` and
  ``unknown`` are the reference's non-transactions (gemini_parser.py:41): every
  other field is null, post-processing raises on ``str(None)`` (:235-241) and the
  worker dead-letters the message as ``{"reason": "unmatched"}`` (worker.py:151-158);
* per copied field, a start row scores every prompt position ``j`` against the
  start-pointer row ``ptr0 + j`` (the same row is added to position ``j``'s input,
  as in the span format, so the model can name a position) and against the
  ``null_id`` row (an empty value); an end row scores position ``j`` against the
  end-pointer row ``pe0 + j``.  With ``n_queries == 9`` one row per field does
  both, with 17 the start and end rows are separate query tokens;
* decoding is joint and constrained: the field is null when its null score is at
  least every valid start's score; otherwise the (start, end) pair maximising
  ``start[s] + end[e]`` over VALID pairs -- ``s <= e < s + cap``, every token in
  the field's class, ``s`` and ``e + 1`` at word boundaries, a date / number never
  starting right after a card mask.  Word boundaries split letters from digits
  ("USD52.00", "x1234" and "1500р" separate), unlike the span format's rule, and
  join a digit group to a lone separator and a three-digit group ("218" "," "993" is
  one word).  Value edges by kind (:data:`EDGE_RULES`): a number starts and ends with
  a digit, a card ends with one, a date or a free-text value starts and ends with a
  letter or digit; no value crosses a line break.  A date span without a time of day
  takes the time token right next to it ("22:09 13.02.2023": the value is a datetime),
  and one ending in digits takes a following AM / PM ("2:23 PM").

The answer is written in the copy format (txn tokens, then each field's body
tokens, each ended by ``<sep>``), so the tokenizers' field decoders, the remote
protocol and post-processing are unchanged.  :func:`qa_decode_ref` is the PyTorch
reference of ``qa_decode_kernel`` (ops/csrc/qa_kernels.hip).
"""
from __future__ import annotations

import re
from dataclasses import dataclass
from typing import Dict, List, Optional, Sequence, Tuple

import numpy as np

from ..parse.schema import TXN_TYPES
from .fsm import DEFAULT_FIELDS, TOK_CLASS_BITS, FieldSpec, _token_class_sets

__all__ = ["QALayout", "qa_layout", "qa_token_flags", "qa_targets", "qa_decode_ref", "qa_expand", "qa_rows", "qa_logits", "qa_loss",
           "REJECT_TXN", "ABSTAIN_TXN", "null_rejection", "qa_confidence", "QF_SL", "QF_SD", "QF_EL", "QF_ED", "QF_MASK", "QA_CLASS_BITS",
           "QA_MAX_QUERIES", "EDGE_RULES", "QF_NL", "QF_FA", "QF_FD", "QF_LA", "QF_LD", "QF_GRP3", "QF_SEP",
           "QF_TIME", "QF_DEND", "QF_AMPM", "QF_AP", "QF_M", "QF_TEXT", "QF_CARDL", "QF_COLON", "QF_XMASK"]

# non-transaction classes: every other field of the answer is null
REJECT_TXN = ("otp", "unknown")
# the class an abstained answer (confidence under the threshold) is turned into: the
# reference's "not a transaction" shape, so the message is dead-lettered as unmatched
ABSTAIN_TXN = "unknown"
QA_MAX_QUERIES = 24
# per-token flags (uint32): starts / ends with a letter / digit, ends a card mask, class bits
QF_SL, QF_SD, QF_EL, QF_ED, QF_MASK = 1, 2, 4, 8, 16
QF_TEXT = 1 << 21  # may be inside a free-text value (merchant / city / address): no ':' in it
# date 32, number 64, currency 128, card 256; text: a label's colon ("Sender: NAME") is never
# part of a name (no gold merchant / city / address of any family has one), so a text value
# never runs across one
QA_CLASS_BITS = {**{k: v << 3 for k, v in TOK_CLASS_BITS.items()}, "text": QF_TEXT}
_NO_START_AFTER_MASK = QA_CLASS_BITS["date"] | QA_CLASS_BITS["number"]
# edges: contains a line break; first non-space char a letter-or-digit / a digit; last
# char a letter-or-digit / a digit; exactly three ASCII digits; a lone "," "." "'"
QF_NL, QF_FA, QF_FD, QF_LA, QF_LD, QF_GRP3, QF_SEP = 512, 1024, 2048, 4096, 8192, 16384, 32768
QF_TIME = 1 << 16  # a whole time of day: " 22:09", "05:27:11"
QF_DEND = 1 << 17  # may end a date: last char a digit, or AM / PM
QF_AMPM = 1 << 18  # " AM" / " PM" as one token
QF_AP = 1 << 19  # " A" / " P": the first piece of a split " AM" / " PM"
QF_M = 1 << 20  # "M": its second piece
# " CARD" + ":" is what normalize_body writes for a "4083***7538" mask ("CARD:7538"): the
# digits after that colon are the card's, so a date or a number never starts there
# (like after a mask); so are digits glued to a token of x / X letters only ("XXXX1438",
# "xx0735": x-masks), but not a spaced word after one ("HSMEX 07 Dec")
QF_CARDL = 1 << 22  # " CARD" / "CARD"
QF_COLON = 1 << 23  # a lone ":"
QF_XMASK = 1 << 24  # x / X letters only
_TIME_RE = re.compile(r" ?\d{1,2}:\d{2}(?::\d{2})?\Z")
# field kind -> (flags its first token must all have, flags its last token must all have).
# A date ends with a digit or AM / PM (a span into the next word -- "12.05.25 покупка",
# month names make letters part of the date class -- is no date).
# Every gold value of every training and held-out family obeys them (a free-text value
# may start with a digit: "7-ELEVEN").
EDGE_RULES = {"number": (QF_FD, QF_LD), "card": (0, QF_LD), "date": (QF_FA, QF_DEND), "text": (QF_FA, QF_LA),
              "currency": (0, 0)}


@dataclass(frozen=True)
class QALayout:
    """Ids of the qa format past the tokenizer's vocabulary (``vocab_tok``)."""
    vocab_tok: int
    n_pos: int  # pointable prompt positions (max_body_tokens + 2)
    n_queries: int  # 9 (one row per field) or 17 (txn + a start and an end row per copied field)
    ptr0: int
    pe0: int
    q0: int
    null_id: int
    cls0: int
    vocab: int  # rounded up to 128
    fields: Tuple[FieldSpec, ...] = DEFAULT_FIELDS

    @property
    def n_copy(self) -> int:
        return len(self.fields) - 1

    def start_row(self, f: int) -> int:
        """Query row scoring copied field ``f``'s start (f = 1 .. n_copy)."""
        return f if self.n_queries == len(self.fields) else 2 * f - 1

    def end_row(self, f: int) -> int:
        return f if self.n_queries == len(self.fields) else 2 * f

    def query_ids(self) -> List[int]:
        return [self.q0 + k for k in range(self.n_queries)]

    def caps(self) -> List[int]:
        return [f.cap for f in self.fields[1:]]

    def class_bits(self) -> List[int]:
        return [QA_CLASS_BITS.get(f.kind, 0) for f in self.fields[1:]]

    def rules(self) -> List[Tuple[int, int, int, int]]:
        """Per copied field: (class bits, cap, first-token edge flags, last-token edge flags)."""
        return [(QA_CLASS_BITS.get(f.kind, 0), f.cap) + EDGE_RULES.get(f.kind, (0, 0)) for f in self.fields[1:]]

    def absorb_time(self) -> List[bool]:
        """Per copied field: a span without a time of day takes an adjacent one (dates)."""
        return [f.kind == "date" for f in self.fields[1:]]

    def max_answer_tokens(self) -> int:
        return sum(f.cap for f in self.fields) + len(self.fields)


def qa_layout(vocab_tok: int = 8192, n_pos: int = 130, n_queries: int = 9,
              fields: Sequence[FieldSpec] = DEFAULT_FIELDS) -> QALayout:
    if fields[0].kind != "enum" or any(f.kind == "enum" or not f.copy for f in fields[1:]):
        raise ValueError("qa format: txn_type enum first, then copied fields")
    if n_queries not in (len(fields), 2 * len(fields) - 1):
        raise ValueError(f"qa format: {len(fields)} or {2 * len(fields) - 1} queries, not {n_queries}")
    ptr0 = vocab_tok
    pe0 = ptr0 + n_pos
    q0 = pe0 + n_pos
    null_id = q0 + QA_MAX_QUERIES
    cls0 = null_id + 1
    vocab = -(-(cls0 + len(TXN_TYPES)) // 128) * 128
    return QALayout(vocab_tok, n_pos, n_queries, ptr0, pe0, q0, null_id, cls0, vocab, tuple(fields))


def qa_token_flags(tokenizer, vocab: int) -> np.ndarray:
    """uint32 per id: QF_* letter / digit start / end bits, card-mask end, class bits."""
    strings = tokenizer.token_strings
    specials = [tokenizer.pad, tokenizer.bos, tokenizer.eos, tokenizer.sep, tokenizer.sms, tokenizer.ans]
    classes = _token_class_sets(strings, specials)
    out = np.zeros(vocab, dtype=np.uint32)
    n = min(vocab, len(strings))
    for k, bit in QA_CLASS_BITS.items():
        out[:n] |= np.where(classes[k][:n], bit, 0).astype(np.uint32)  # text: every non-special token
    no_text = np.uint32(~QF_TEXT & 0xFFFFFFFF)
    spec = set(specials)

    def letter(ch: str) -> bool:
        return ch.isalpha() or ch == "�"

    for i, t in enumerate(strings[:vocab]):
        if i in spec or not t:
            continue
        f = 0
        if letter(t[0]):
            f |= QF_SL
        # a number's inner separator before a digit continues the number (".58" of "657.58")
        if t[0].isdigit() or (len(t) > 1 and t[0] in ".,:'" and t[1].isdigit()):
            f |= QF_SD
        if letter(t[-1]):
            f |= QF_EL
        if t[-1].isdigit() or (len(t) > 1 and t[-1] in ".,:'" and t[-2].isdigit()):
            f |= QF_ED
        if t.endswith("*"):
            f |= QF_MASK
        if t.strip(" ") and not t.strip(" ").strip("xX"):
            f |= QF_XMASK
        if t.strip(" ") == "CARD":
            f |= QF_CARDL
        if t == ":":
            f |= QF_COLON
        if "\n" in t:
            f |= QF_NL
        h = t.lstrip(" ")
        if h and (h[0].isalnum() or h[0] == "�"):
            f |= QF_FA
        if h[:1].isdigit():
            f |= QF_FD
        if t[-1].isalnum() or t[-1] == "�":
            f |= QF_LA
        if t[-1].isdigit():
            f |= QF_LD
        if len(t) == 3 and t.isascii() and t.isdigit():
            f |= QF_GRP3
        if t in (",", ".", "'"):
            f |= QF_SEP
        if _TIME_RE.match(t):
            f |= QF_TIME
        if t[-1].isdigit() or t.strip().upper() in ("AM", "PM", "M"):  # "PM" is " P" + "M"
            f |= QF_DEND
        if t.upper() in (" AM", " PM"):
            f |= QF_AMPM
        if t.upper() in (" A", " P"):
            f |= QF_AP
        if t.upper() == "M":
            f |= QF_M
        out[i] |= f
        if ":" in t:
            out[i] &= no_text
    return out


def _glued(fa: int, fb: int) -> bool:
    return bool(((fa & QF_EL) and (fb & QF_SL)) or ((fa & QF_ED) and (fb & QF_SD)))


def _fl(flags: np.ndarray, body: Sequence[int], j: int) -> int:
    return int(flags[body[j]])


def _start_ok(flags, body, j: int, cls: int, s_need: int) -> bool:
    fj = _fl(flags, body, j)
    if (cls and not fj & cls) or fj & QF_NL or (fj & s_need) != s_need:
        return False
    if j > 0:
        fp = _fl(flags, body, j - 1)
        if _glued(fp, fj) or ((cls & _NO_START_AFTER_MASK) and fp & QF_MASK):
            return False
        if (cls & _NO_START_AFTER_MASK) and ((fp & QF_XMASK and fj & QF_SD) or (
                j > 1 and fp & QF_COLON and _fl(flags, body, j - 2) & QF_CARDL)):
            return False  # "1438" of "XXXX1438", "7538" of "CARD:7538"
        if j > 1 and fp & QF_SEP and fj & QF_GRP3 and _fl(flags, body, j - 2) & QF_LD:
            return False  # "993" of "218,993"
    return True


def _end_ok(flags, body, n: int, e: int, e_need: int) -> bool:
    fe = _fl(flags, body, e)
    if (fe & e_need) != e_need:
        return False
    if e + 1 < n and (_glued(fe, _fl(flags, body, e + 1)) or (
            e > 0 and fe & QF_SEP and _fl(flags, body, e + 1) & QF_GRP3 and _fl(flags, body, e - 1) & QF_LD)):
        return False
    if e + 2 < n and fe & QF_LD and _fl(flags, body, e + 1) & QF_SEP and _fl(flags, body, e + 2) & QF_GRP3:
        return False  # "218" of "218,993"
    return True


def valid_starts(flags: np.ndarray, body: Sequence[int], n: int, cls: int, s_need: int = 0) -> np.ndarray:
    """[n] bool: positions a value of class bits ``cls`` may start at (``n`` pointable);
    ``s_need``: flags the first token must all have (:data:`EDGE_RULES`)."""
    return np.array([_start_ok(flags, body, j, cls, s_need) for j in range(n)], dtype=bool)


def valid_ends(flags: np.ndarray, body: Sequence[int], n: int, cls: int, cap: int, s: int,
               e_need: int = 0) -> List[int]:
    """End positions of a value starting at ``s``: in class all the way and never across
    a line break, within the cap, with the last token's edge flags ``e_need``, followed
    by a word boundary (or the end of the pointable body)."""
    out = []
    for e in range(s, min(n, s + cap)):
        fe = _fl(flags, body, e)
        if (cls and not fe & cls) or fe & QF_NL:
            break
        if _end_ok(flags, body, n, e, e_need):
            out.append(e)
    return out


def qa_targets(tok, lay: QALayout, flags: np.ndarray, answer: Dict[str, Optional[str]], body: str, body_enc,
               msg_len: int) -> Optional[Tuple[int, List[Tuple[int, int]]]]:
    """Training target ``(class index, [(start, end) | (-1, -1) per copied field])`` or
    None when a gold value is not a valid span the decoder could produce (the span
    format's answer_span_tokens drops such examples too)."""
    txn = answer.get("txn_type") or "unknown"
    if txn not in TXN_TYPES:
        return None
    cls = TXN_TYPES.index(txn)
    n = msg_len - 1  # pointable positions (the message ends with <ans>)
    ids = body_enc[0]
    spans: List[Tuple[int, int]] = []
    for f, (bits, cap, s_need, e_need) in zip(lay.fields[1:], lay.rules()):
        v = answer.get(f.name) or ""
        if not v or txn in REJECT_TXN:
            spans.append((-1, -1))
            continue
        sp = tok.value_span(v, body, ids, body_enc[1])
        if sp is None or sp[1] >= n:
            return None
        s, e = sp
        if not _start_ok(flags, ids, s, bits, s_need) or e not in valid_ends(flags, ids, n, bits, cap, s, e_need):
            return None
        spans.append((s, e))
    return cls, spans


def qa_rows(lay: QALayout) -> Tuple[List[int], List[int]]:
    """(start row, end row) per copied field."""
    return ([lay.start_row(f) for f in range(1, len(lay.fields))],
            [lay.end_row(f) for f in range(1, len(lay.fields))])


def _pair_mask(fb: np.ndarray, n: int, cls: int, cap: int, s_need: int = 0,
               e_need: int = 0) -> Tuple[np.ndarray, np.ndarray]:
    """(valid starts [n], valid (start, end) pairs [n, n]) of one field from the body's
    token flags ``fb`` (vectorised :func:`valid_starts` / :func:`valid_ends`)."""
    fb = fb[:n].astype(np.int64)
    prev = np.concatenate([[0], fb[:-1]])
    prev2 = np.concatenate([[0, 0], fb[:-2]])[:n]
    glued_prev = (((prev & QF_EL) != 0) & ((fb & QF_SL) != 0)) | (((prev & QF_ED) != 0) & ((fb & QF_SD) != 0))
    glued_prev |= ((prev & QF_SEP) != 0) & ((fb & QF_GRP3) != 0) & ((prev2 & QF_LD) != 0)
    glued_prev[0] = False
    in_cls = (fb & cls) != 0 if cls else np.ones(n, dtype=bool)
    in_cls &= (fb & QF_NL) == 0
    after_mask = (((prev & QF_MASK) != 0) | (((prev & QF_COLON) != 0) & ((prev2 & QF_CARDL) != 0))
                  | (((prev & QF_XMASK) != 0) & ((fb & QF_SD) != 0))) & bool(cls & _NO_START_AFTER_MASK)
    after_mask[0] = False
    vs = in_cls & ~glued_prev & ~after_mask & ((fb & s_need) == s_need)
    # an end may not be followed by a glued token, nor by a separator glued to a group
    end_ok = (fb & e_need) == e_need
    end_ok[:-1] &= ~glued_prev[1:]
    nxt_sep = np.zeros(n, dtype=bool)
    nxt_sep[:-2] = ((fb[:-2] & QF_LD) != 0) & ((fb[1:-1] & QF_SEP) != 0) & ((fb[2:] & QF_GRP3) != 0)
    end_ok &= ~nxt_sep
    bad = np.concatenate([[0], np.cumsum(~in_cls)])  # out-of-class tokens before position k
    S, E = np.arange(n)[:, None], np.arange(n)[None, :]
    pairs = (E >= S) & (E - S < cap) & (bad[E + 1] - bad[S] == 0) & end_ok[None, :] & vs[:, None]
    return vs, pairs


def _absorb_time(fb: np.ndarray, pairs: np.ndarray, a: int, z: int, n: int) -> Tuple[int, int]:
    """A date span (a, z) with no time-of-day token takes the one right before it, else
    the one right after it, when the longer span is itself a valid pair; then a span
    ending in a digit takes a following " AM" / " PM" (one token or " A" / " P" + "M")."""
    if not (fb[a:z + 1] & QF_TIME).any():
        if a > 0 and fb[a - 1] & QF_TIME and pairs[a - 1, z]:
            a -= 1
        elif z + 1 < n and fb[z + 1] & QF_TIME and pairs[a, z + 1]:
            z += 1
    if fb[z] & QF_LD:
        if z + 1 < n and fb[z + 1] & QF_AMPM and pairs[a, z + 1]:
            z += 1
        elif z + 2 < n and fb[z + 1] & QF_AP and fb[z + 2] & QF_M and pairs[a, z + 2]:
            z += 2
    return a, z


def _p_of(logits: np.ndarray, k: int) -> float:
    """Softmax probability of entry ``k`` (fp32, max-shifted like the kernel)."""
    x = np.asarray(logits, dtype=np.float32)
    mx = x.max()
    return float(np.exp(x[k] - mx) / np.exp(x - mx).sum(dtype=np.float32))


def qa_confidence(cls_logits, start_logits, null_logits, end_logits, n: int, c: int,
                  spans: Sequence[Tuple[int, int]]) -> float:
    """An answer's confidence: the probability of its least probable decision under the
    head's training distributions (:func:`qa_loss`) -- the class softmax; per copied
    field the start softmax over the ``n`` body positions and null (for a null field the
    null probability) times the end softmax over the body positions.  ``spans``: the
    decoded (start, end) BEFORE time / AM-PM absorption; a rejection is judged by its
    class alone."""
    conf = _p_of(cls_logits, c)
    if TXN_TYPES[c] in REJECT_TXN:
        return conf
    for f, (a, z) in enumerate(spans):
        st = np.concatenate([np.asarray(start_logits[f][:n], dtype=np.float32),
                             np.asarray([null_logits[f]], dtype=np.float32)])
        if a < 0:
            pf = _p_of(st, n)
        else:
            pf = _p_of(st, a) * _p_of(np.asarray(end_logits[f][:n], dtype=np.float32), z)
        conf = min(conf, pf)
    return conf


def qa_decode_ref(cls_logits, start_logits, null_logits, end_logits, bodies: Sequence[Sequence[int]],
                  flags: np.ndarray, lay: QALayout, min_conf: float = 0.0,
                  conf_out: Optional[List[float]] = None) -> List[Tuple[int, List[Tuple[int, int]]]]:
    """Reference joint decode (host, numpy).  Per message ``m``: ``cls_logits[m]`` [4],
    ``start_logits[m]`` / ``end_logits[m]`` [n_copy, >= n] over prompt positions,
    ``null_logits[m]`` [n_copy]; ``bodies[m]`` the prompt ids (``body <ans>``).
    Returns (class, spans) with (-1, -1) for a null field (every field of a rejection).
    Ties go to the lower class, then the lower start, then the lower end (the kernel's
    rule); the field is null when its null score is >= every valid start's score or no
    valid pair exists.  A transaction answer whose :func:`qa_confidence` is under
    ``min_conf`` abstains: class :data:`ABSTAIN_TXN`, every field null.  ``conf_out``
    collects each answer's confidence (before abstention)."""
    out = []
    abstain = TXN_TYPES.index(ABSTAIN_TXN)
    for m, body in enumerate(bodies):
        c = int(np.argmax(np.asarray(cls_logits[m], dtype=np.float32)))
        if TXN_TYPES[c] in REJECT_TXN:
            if conf_out is not None:
                conf_out.append(_p_of(cls_logits[m], c))
            out.append((c, [(-1, -1)] * lay.n_copy))
            continue
        n = len(body) - 1
        fb = flags[np.asarray(body[:n], dtype=np.int64)]
        spans: List[Tuple[int, int]] = []
        raw: List[Tuple[int, int]] = []  # before absorption: what the confidence judges
        absorb = lay.absorb_time()
        for f, (bits, cap, s_need, e_need) in enumerate(lay.rules()):
            st = np.asarray(start_logits[m][f][:n], dtype=np.float32)
            en = np.asarray(end_logits[m][f][:n], dtype=np.float32)
            vs, pairs = _pair_mask(fb, n, bits, cap, s_need, e_need)
            if not pairs.any() or np.float32(null_logits[m][f]) >= st[vs].max():
                spans.append((-1, -1))
                raw.append((-1, -1))
                continue
            sc = np.where(pairs, st[:, None] + en[None, :], -np.inf)
            k = int(np.argmax(sc))
            a, z = k // n, k % n
            raw.append((a, z))
            if absorb[f]:
                a, z = _absorb_time(fb, pairs, a, z, n)
            spans.append((a, z))
        conf = qa_confidence(cls_logits[m], start_logits[m], null_logits[m], end_logits[m], n, c, raw)
        if conf_out is not None:
            conf_out.append(conf)
        if conf < min_conf:
            out.append((abstain, [(-1, -1)] * lay.n_copy))
            continue
        out.append((c, spans))
    return out


def qa_expand(tok, lay: QALayout, cls: int, spans: Sequence[Tuple[int, int]], body: Sequence[int]) -> List[int]:
    """The copy-format answer tokens of a decoded (class, spans)."""
    out = list(tok.encode(TXN_TYPES[cls])) + [tok.sep]
    if TXN_TYPES[cls] in REJECT_TXN:
        return out
    for s, e in spans:
        if s >= 0:
            out += list(body[s:e + 1])
        out.append(tok.sep)
    return out


def qa_logits(h, embed, qpos, lay: QALayout):
    """Scores of the query rows (PyTorch; training and the reference path).  ``h`` [B, T, H]
    final-normed hidden states, ``embed`` the (tied) embedding, ``qpos`` [B, n_queries]
    the query rows' positions.  Returns fp32 ``cls`` [B, 4], ``start`` [B, n_copy, n_pos],
    ``null`` [B, n_copy], ``end`` [B, n_copy, n_pos]."""
    import torch

    B = h.shape[0]
    hq = h[torch.arange(B, device=h.device)[:, None], qpos]  # [B, NQ, H]
    srows, erows = qa_rows(lay)
    hs, he = hq[:, srows], hq[:, erows]
    E = embed if embed.dtype == h.dtype or torch.is_autocast_enabled() else embed.to(h.dtype)
    cls = (hq[:, 0] @ E[lay.cls0:lay.cls0 + len(TXN_TYPES)].t()).float()
    start = (hs @ E[lay.ptr0:lay.ptr0 + lay.n_pos].t()).float()
    null = (hs @ E[lay.null_id]).float()
    end = (he @ E[lay.pe0:lay.pe0 + lay.n_pos].t()).float()
    return cls, start, null, end


def qa_loss(scores, targets, lay: QALayout, denom: Optional[float] = None):
    """Mean cross-entropy over the answer's decisions: the class, every copied field's
    start (null included) and every non-null field's end (over all message positions).
    ``targets``: (cls [B], starts [B, n_copy] (-1 = null), ends [B, n_copy], npos [B]
    pointable positions per message).  ``denom``: the decision count to divide by, from
    the host (no device sync; data parallel: the GLOBAL batch's count / world, so the
    averaged gradient is the one-GPU batch's); default this batch's own count."""
    import torch
    import torch.nn.functional as F

    cls, start, null, end = scores
    t_cls, t_s, t_e, npos = targets
    B, NF, NP = start.shape
    j = torch.arange(NP, device=start.device)
    out_of_msg = j[None, None, :] >= npos[:, None, None]  # [B, 1, NP]
    neg = torch.finfo(torch.float32).min / 4
    st = torch.cat([start.masked_fill(out_of_msg, neg), null[..., None]], -1)  # null = index NP
    st_t = torch.where(t_s >= 0, t_s, torch.full_like(t_s, NP))
    l_cls = F.cross_entropy(cls, t_cls, reduction="sum")
    l_st = F.cross_entropy(st.reshape(-1, NP + 1), st_t.reshape(-1), reduction="sum")
    has = t_s >= 0
    # the end distribution is trained over EVERY position of the message, not only those
    # at / after the gold start: the decoder scores (start, end) pairs jointly, and end
    # scores left untrained before the start would let a wrong pair win
    en = end.masked_fill(out_of_msg, neg)
    l_en = F.cross_entropy(en[has], t_e[has], reduction="sum") if bool(has.any()) else en.sum() * 0
    return (l_cls + l_st + l_en) / (denom if denom is not None else (B + B * NF + int(has.sum())))


def null_rejection(answer: Dict[str, Optional[str]]) -> Dict[str, Optional[str]]:
    """A decoded answer whose txn_type is a non-transaction gets null fields (Gemini's
    shape for "not a transaction"): post-processing then raises on ``str(None)`` and
    the message is dead-lettered as unmatched, the reference's path."""
    if answer.get("txn_type") in REJECT_TXN:
        return {k: (v if k == "txn_type" else None) for k, v in answer.items()}
    return answer
