"""Schema finite-state machine for constrained extraction decoding.

The reference asks Gemini for JSON matching a 9-key schema
(gemini_parser.py:46-61, ``response_mime_type=application/json``). The local
extractor instead emits the nine values in schema order, each terminated by
``<sep>`` — the JSON scaffolding (keys, quotes, braces) is implied by the
schema, so no decode step is spent on it. Every step is constrained by this
FSM, compiled into GPU tables and applied inside ``sg_fsm_sample``:

* a **value state** ``(field, k)`` allows the field's token class plus
  ``<sep>``; at the field's token cap only ``<sep>`` is allowed, so every
  sequence terminates within ``sum(caps) + 9`` steps;
* ``txn_type`` is an **enum** compiled to a token trie over the tokenizer's
  encodings of ``debit | credit | otp | unknown``;
* token classes are derived from each token's decoded text (digits/dots for
  dates, digits/separators for amounts, capitals for currencies, …).

Tables (``int32``/``uint32`` on the device): ``masks[S, V/32]`` allowed-token
bitmasks, ``next_sep[S]``, ``next_tok[S]`` (``-2`` = look up the sparse enum
table ``enum_tok/enum_next[S, E]``), plus ``done_state``.
"""
from __future__ import annotations

from dataclasses import dataclass, field
from typing import Dict, List, Optional, Sequence, Tuple

import numpy as np

from ..models.domain import CORE_FIELDS
from ..parse.schema import TXN_TYPES

__all__ = ["FieldSpec", "SchemaFSM", "DEFAULT_FIELDS", "build_fsm", "build_span_fsm", "COPY_NONE", "COPY_START",
           "COPY_NEXT", "PTR_START", "PTR_END", "TOK_STARTS_ALNUM", "TOK_ENDS_ALNUM", "token_flags", "span_positions"]


@dataclass(frozen=True)
class FieldSpec:
    name: str
    kind: str  # text | date | number | currency | card | enum
    cap: int
    choices: Tuple[str, ...] = ()
    # copy-constrained: every value token is a token of the SMS body, and after the
    # first one each token must follow the previous one at some body position; a
    # value starts and ends at a word boundary of the body (never inside a word
    # split into several tokens) -- COPY_START / COPY_NEXT states, masks built per
    # row by ops.copy_masks
    copy: bool = False


# Token caps per field.  Measured on 20 k synthetic SMS of each vocabulary and of the
# template families (utils/synth.py) with the extractor tokenizer (values written with
# the body's own tokens): max tokens seen date 9, amount/balance 6, currency 2, card 3,
# merchant 32, city 14 (Cyrillic names split into byte-level pieces), address 16
# (tests/test_fsm_caps.py pins a truncation rate of 0 on held-out data,
# tests/test_families.py that no family uses more than ~3/4 of a cap).  The caps
# are about 1.5-2x those maxima (the total keeps Lmax at 288 KV positions per slot):
# a cap only bounds the KV length reserved per slot
# (rows stop at <sep>, so decode cost does not depend on it), and a value longer
# than its cap would be silently cut.
#
# Every non-enum value is copied from the body (the reference's golden answers are
# substrings of their SMS, tests/test_parsers.py:11-58; all synthetic gold values are
# token-aligned body spans, tests/test_copy_fsm.py), so every non-enum field is
# copy-constrained: the model can pick the span, never invent a name.
DEFAULT_FIELDS: Tuple[FieldSpec, ...] = (
    FieldSpec("txn_type", "enum", 8, TXN_TYPES),  # cap = bound on the enum trie depth
    FieldSpec("date", "date", 20, copy=True),  # "11 февраля 2025 г. 11:54": 14 tokens
    FieldSpec("amount", "number", 10, copy=True),
    FieldSpec("currency", "currency", 4, copy=True),
    FieldSpec("card", "card", 6, copy=True),
    FieldSpec("merchant", "text", 48, copy=True),
    FieldSpec("city", "text", 20, copy=True),
    FieldSpec("address", "text", 24, copy=True),
    FieldSpec("balance", "number", 10, copy=True),
)
assert tuple(f.name for f in DEFAULT_FIELDS) == CORE_FIELDS

# per-state copy kind (SchemaFSM.copy_kind; low byte).  The span-pointer format's end
# state also carries the field's token cap (bits 8-15) and token-class bit (16-23)
COPY_NONE, COPY_START, COPY_NEXT, PTR_START, PTR_END = 0, 1, 2, 3, 4
# per-token flags (SchemaFSM.tok_flags): the token's text starts / ends with a letter or
# digit.  Between body tokens a and b there is a word boundary unless a ends and b
# starts alphanumeric (b then continues a's word: byte-level BPE puts the blank in b)
TOK_STARTS_ALNUM, TOK_ENDS_ALNUM = 1, 2
# token-class bits (span format: every token of a pointed-to span must be in the
# field's class, as every copied token must be in copy format's schema mask)
TOK_CLASS_BITS = {"date": 4, "number": 8, "currency": 16, "card": 32}
# the token closes a card mask ("****", " *"): the digits after it are the card's, so a
# date or a number never starts right after it (span format; "**** 7492 17.05.24" is not
# the date "7492 17.05.24")
TOK_ENDS_MASK = 64
_NO_START_AFTER_MASK = TOK_CLASS_BITS["date"] | TOK_CLASS_BITS["number"]


def token_flags(token_strings: Sequence[str], specials: Sequence[int], vocab: int,
                classes: Optional[Dict[str, np.ndarray]] = None) -> np.ndarray:
    out = np.zeros(vocab, dtype=np.uint8)
    spec = set(specials)
    if classes is not None:
        n = min(vocab, len(token_strings))
        for k, bit in TOK_CLASS_BITS.items():
            out[:n] |= np.where(classes[k][:n], bit, 0).astype(np.uint8)
    for i, t in enumerate(token_strings[:vocab]):
        if i in spec or not t:
            continue
        # a byte-level piece of a multi-byte character decodes to U+FFFD: it is inside a
        # word (Cyrillic letters), never a word boundary.  A token that opens with a
        # number's inner separator followed by a digit (".58", ",000", ":23") continues
        # the number before it like a letter continues a word: a value can neither start
        # there ("657.58" -> "0.58") nor end just before it ("657" of "657.58")
        # (and likewise a token that closes with one after a digit, " 1," of "1,234.50")
        starts = t[0].isalnum() or t[0] == "\ufffd" or (len(t) > 1 and t[0] in ".,:" and t[1].isdigit())
        ends = t[-1].isalnum() or t[-1] == "\ufffd" or (len(t) > 1 and t[-1] in ".,:" and t[-2].isdigit())
        out[i] |= (TOK_STARTS_ALNUM if starts else 0) | (TOK_ENDS_ALNUM if ends else 0) | \
            (TOK_ENDS_MASK if t.endswith("*") else 0)
    return out

# token classes by the characters of a token's text.  Dates may carry ASCII letters
# (month names "10 Jun 2025", the ISO "T"); currencies are codes, symbols or words in
# any script ("USD", "$", "руб") -- parse/canonical.py maps the last two to ISO codes
_ASCII_LETTERS = set("ABCDEFGHIJKLMNOPQRSTUVWXYZabcdefghijklmnopqrstuvwxyz")
_CURRENCY_SYMBOLS = set("$€£₽₾֏")
_CYRILLIC = set("абвгдеёжзийклмнопрстуфхцчшщъыьэюяАБВГДЕЁЖЗИЙКЛМНОПРСТУФХЦЧШЩЪЫЬЭЮЯ") | {"�"}
_CLASS_CHARS = {
    # month names in Latin or Cyrillic script ("6 июня 2025"; byte-level pieces of a
    # Cyrillic letter decode to U+FFFD)
    "date": set("0123456789.:/-, ") | _ASCII_LETTERS | _CYRILLIC,
    # apostrophe / right single quote thousands ("1'234.56", Swiss style)
    "number": set("0123456789.,- '’"),
    "currency": {" "} | _CURRENCY_SYMBOLS,  # plus any alphabetic character (below)
    "card": set("0123456789* "),
}


def _token_class_sets(token_strings: Sequence[str], specials: Sequence[int]) -> Dict[str, np.ndarray]:
    V = len(token_strings)
    spec = set(specials)
    out = {k: np.zeros(V, dtype=bool) for k in ("text", "date", "number", "currency", "card")}
    for i, s in enumerate(token_strings):
        if i in spec or not s:
            continue
        out["text"][i] = True
        if not s.strip():
            # pure-whitespace tokens only count as free text -- except one blank inside a
            # date: byte-level BPE leaves the blank before a Cyrillic month name alone
            # (" 18", " ", "я", "н", ... of "18 января")
            out["date"][i] = s == " "
            continue
        cs = set(s)
        for k, allowed in _CLASS_CHARS.items():
            if cs <= allowed or (k == "currency" and all(ch in allowed or ch.isalpha() for ch in cs)):
                out[k][i] = True
    return out


@dataclass
class SchemaFSM:
    fields: Tuple[FieldSpec, ...]
    vocab: int  # model vocab (≥ tokenizer vocab; extra ids never allowed)
    sep_token: int
    allowed: np.ndarray  # [S, vocab] bool
    next_sep: np.ndarray  # [S]
    next_tok: np.ndarray  # [S] (-2 = enum lookup)
    enum_tok: np.ndarray  # [S, E]
    enum_next: np.ndarray  # [S, E]
    done_state: int
    start_state: int = 0
    field_of_state: List[int] = field(default_factory=list)
    copy_kind: Optional[np.ndarray] = None  # [S] COPY_NONE / COPY_START / COPY_NEXT (| PTR_* for spans)
    tok_flags: Optional[np.ndarray] = None  # [vocab] uint8 TOK_STARTS_ALNUM | TOK_ENDS_ALNUM (| class bits)
    # span-pointer format (build_span_fsm): pointer token ptr0 + j = body position j
    ptr0: int = -1
    n_pos: int = 0
    # device copies (filled by to_device; consumed by ops.fsm_sample)
    masks: object = None
    state_mask: object = None
    next_sep_t: object = None
    next_tok_t: object = None
    enum_tok_t: object = None
    enum_next_t: object = None
    forced_t: object = None
    copy_kind_t: object = None
    tok_flags_t: object = None

    @property
    def has_copy(self) -> bool:
        return self.copy_kind is not None and bool((self.copy_kind != COPY_NONE).any())

    @property
    def forced(self) -> np.ndarray:
        """[S] the only token a state allows (-1: several, or the done state)."""
        one = self.allowed.sum(1) == 1
        out = np.where(one, self.allowed.argmax(1), -1).astype(np.int32)
        out[self.done_state] = -1
        return out

    @property
    def E(self) -> int:
        return int(self.enum_tok.shape[1])

    @property
    def num_states(self) -> int:
        return int(self.allowed.shape[0])

    @property
    def span(self) -> bool:
        return self.ptr0 >= 0

    def max_steps(self) -> int:
        """Decode steps (= KV positions) an answer can take."""
        if self.span:
            return sum(f.cap + 1 if f.kind == "enum" else 2 for f in self.fields)
        return self.max_answer_tokens()

    def max_answer_tokens(self) -> int:
        """Length of the longest answer in copy format (the span format's answers are
        expanded to it on the GPU: ops.span_commit)."""
        return sum(f.cap for f in self.fields) + len(self.fields)

    def packed_masks(self) -> np.ndarray:
        """[S, vocab/32] uint32, bit j of word w = token 32w+j allowed."""
        S, V = self.allowed.shape
        bits = self.allowed.reshape(S, V // 32, 32).astype(np.uint64)
        weights = (np.uint64(1) << np.arange(32, dtype=np.uint64))
        return (bits * weights).sum(-1).astype(np.uint32)

    def to_device(self, device) -> "SchemaFSM":
        import torch

        self.masks = torch.from_numpy(self.packed_masks().view(np.int32)).to(device)
        self.state_mask = torch.arange(self.num_states, dtype=torch.int32, device=device)
        # kernel-facing names
        self.next_sep_t = torch.from_numpy(self.next_sep.astype(np.int32)).to(device)
        self.next_tok_t = torch.from_numpy(self.next_tok.astype(np.int32)).to(device)
        self.enum_tok_t = torch.from_numpy(self.enum_tok.astype(np.int32)).to(device)
        self.enum_next_t = torch.from_numpy(self.enum_next.astype(np.int32)).to(device)
        self.forced_t = torch.from_numpy(self.forced).to(device)
        ck = self.copy_kind if self.copy_kind is not None else np.zeros(self.num_states, dtype=np.int32)
        self.copy_kind_t = torch.from_numpy(ck.astype(np.int32)).to(device)
        tf = self.tok_flags if self.tok_flags is not None else np.zeros(self.vocab, dtype=np.uint8)
        self.tok_flags_t = torch.from_numpy(tf.astype(np.uint8)).to(device)
        return self

    def _boundary(self, a: int, b: int) -> bool:
        """A word boundary between adjacent body tokens ``a`` and ``b``."""
        tf = self.tok_flags
        if tf is None:
            return True
        fa = int(tf[a]) if 0 <= a < self.vocab else 0
        fb = int(tf[b]) if 0 <= b < self.vocab else 0
        return not ((fa & TOK_ENDS_ALNUM) and (fb & TOK_STARTS_ALNUM))

    def copy_mask_host(self, state: int, prev: int, body: Sequence[int]) -> np.ndarray:
        """Reference of ops.copy_masks for one row (tests): [vocab] bool allowed tokens
        of ``state`` after ``prev`` for a row whose prompt ids are ``body``."""
        allow = self.allowed[state].copy()
        kind = COPY_NONE if self.copy_kind is None else int(self.copy_kind[state])
        if kind == COPY_NONE:
            return allow
        if kind & 0xFF in (PTR_START, PTR_END):
            return allow & self._span_candidates(kind, prev, body)
        cand = np.zeros(self.vocab, dtype=bool)
        if kind == COPY_START:
            # a value starts at a word boundary; an empty value (<sep>) is always possible
            for j, t in enumerate(body):
                if 0 <= t < self.vocab and (j == 0 or self._boundary(body[j - 1], t)):
                    cand[t] = True
            cand[self.sep_token] = True
        else:
            # continue along a body bigram; end (<sep>) only where the body has a word boundary
            for j, t in enumerate(body):
                if t != prev:
                    continue
                nxt = body[j + 1] if j + 1 < len(body) else -1
                if 0 <= nxt < self.vocab:
                    cand[nxt] = True
                if nxt < 0 or self._boundary(t, nxt):
                    cand[self.sep_token] = True
        return allow & cand

    def _span_candidates(self, kind: int, prev: int, body: Sequence[int]) -> np.ndarray:
        """Span format (sparse_argmax_kernel's kinds 3 / 4): a start pointer at a word
        boundary whose token is in the field's class, or <sep> (empty value); an end
        pointer e >= start, within the field's cap, every token start..e in the class,
        at a word boundary.  ``body`` ends with <ans>, which is never pointed at."""
        cand = np.zeros(self.vocab, dtype=bool)
        tf = self.tok_flags
        cls = (kind >> 16) & 0xFF
        n = len(body) - 1  # the pointable positions (the last prompt token is <ans>)

        def in_cls(t: int) -> bool:
            return cls == 0 or bool(int(tf[t]) & cls) if 0 <= t < self.vocab else False

        cap = (kind >> 8) & 0xFF

        def ends(s: int) -> List[int]:
            out = []
            for e in range(s, min(n, s + cap)):
                if not in_cls(body[e]):
                    break
                if e + 1 >= n or self._boundary(body[e], body[e + 1]):
                    out.append(e)
            return out

        if kind & 0xFF == PTR_START:
            cand[self.sep_token] = True
            no_mask = bool(cls & _NO_START_AFTER_MASK)
            for j in range(min(n, self.n_pos)):
                # a start must have an end (the end state has no <sep>); an FSM
                # whose start states carry no cap (cap 0) skips the check
                if (j == 0 or self._boundary(body[j - 1], body[j])) and in_cls(body[j]) and \
                        not (no_mask and j > 0 and 0 <= body[j - 1] < self.vocab and tf[body[j - 1]] & TOK_ENDS_MASK) \
                        and (cap == 0 or ends(j)):
                    cand[self.ptr0 + j] = True
            return cand
        s = prev - self.ptr0
        if not 0 <= s < n:
            return cand
        for e in ends(s):
            cand[self.ptr0 + e] = True
        return cand

    def expand_span_answer(self, toks: Sequence[int], body: Sequence[int]) -> List[int]:
        """Span answer -> the copy-format token stream (what ops.span_commit writes)."""
        out: List[int] = []
        st = self.start_state
        start = -1
        for t in toks:
            kind = int(self.copy_kind[st]) & 0xFF if self.copy_kind is not None else 0
            if kind == PTR_END:
                out += list(body[start:t - self.ptr0 + 1]) + [self.sep_token]
            elif kind == PTR_START:
                if t == self.sep_token:
                    out.append(t)
                else:
                    start = t - self.ptr0
            else:
                out.append(t)
            st = self.step_host(st, t)
            if st < 0:
                break
        return out

    def step_host(self, state: int, tok: int) -> int:
        """Reference transition (host side, for tests)."""
        if not self.allowed[state, tok]:
            return -1
        if tok == self.sep_token:
            return int(self.next_sep[state])
        nt = int(self.next_tok[state])
        if nt != -2:
            return nt
        for t, n in zip(self.enum_tok[state], self.enum_next[state]):
            if int(t) == tok:
                return int(n)
        return -1

    def split_fields(self, tokens: Sequence[int]) -> List[List[int]]:
        vals: List[List[int]] = [[]]
        for t in tokens:
            if t == self.sep_token:
                vals.append([])
            else:
                vals[-1].append(t)
        return vals[: len(self.fields)]


def build_fsm(tokenizer, vocab: int, fields: Sequence[FieldSpec] = DEFAULT_FIELDS) -> SchemaFSM:
    strings = tokenizer.token_strings
    V_tok = len(strings)
    specials = [tokenizer.pad, tokenizer.bos, tokenizer.eos, tokenizer.sep, tokenizer.sms, tokenizer.ans]
    classes = _token_class_sets(strings, specials)
    sep = tokenizer.sep

    states_allowed: List[np.ndarray] = []
    next_sep: List[int] = []
    next_tok: List[int] = []
    enum_lists: List[List[Tuple[int, int]]] = []
    field_of: List[int] = []
    copy_kind: List[int] = []

    def new_state(allowed: np.ndarray, fidx: int, ck: int = COPY_NONE) -> int:
        states_allowed.append(allowed)
        next_sep.append(-1)
        next_tok.append(-1)
        enum_lists.append([])
        field_of.append(fidx)
        copy_kind.append(ck)
        return len(states_allowed) - 1

    def pad(mask: np.ndarray) -> np.ndarray:
        full = np.zeros(vocab, dtype=bool)
        full[:V_tok] = mask
        return full

    only_sep = np.zeros(vocab, dtype=bool)
    only_sep[sep] = True

    field_starts: List[int] = []
    field_ends: List[List[int]] = []  # states whose <sep> leaves the field
    for fi, f in enumerate(fields):
        if f.kind == "enum":
            enc = [tokenizer.encode(c) for c in f.choices]
            if max(len(e) for e in enc) > f.cap:
                raise ValueError(f"enum field {f.name!r}: a choice needs more than cap={f.cap} tokens")
            # trie over token sequences
            root = new_state(np.zeros(vocab, dtype=bool), fi)
            field_starts.append(root)
            ends: List[int] = []
            nodes: Dict[Tuple[int, ...], int] = {(): root}
            for seq in enc:
                for depth in range(len(seq)):
                    pre = tuple(seq[:depth])
                    cur = nodes[pre]
                    nxt_key = tuple(seq[: depth + 1])
                    if nxt_key not in nodes:
                        nodes[nxt_key] = new_state(np.zeros(vocab, dtype=bool), fi)
                    states_allowed[cur][seq[depth]] = True
                    if (seq[depth], nodes[nxt_key]) not in enum_lists[cur]:
                        enum_lists[cur].append((seq[depth], nodes[nxt_key]))
                    next_tok[cur] = -2
                leaf = nodes[tuple(seq)]
                states_allowed[leaf][sep] = True
                ends.append(leaf)
            field_ends.append(ends)
        else:
            cls = pad(classes[f.kind])
            allow = cls.copy()
            allow[sep] = True
            st = [new_state(allow.copy(), fi, (COPY_START if k == 0 else COPY_NEXT) if f.copy else COPY_NONE)
                  for k in range(f.cap)]
            last = new_state(only_sep.copy(), fi)
            chain = st + [last]
            for a, b in zip(chain[:-1], chain[1:]):
                next_tok[a] = b
            field_starts.append(chain[0])
            field_ends.append(chain)
    done = new_state(only_sep.copy(), len(fields))
    next_sep[done] = done
    for fi in range(len(fields)):
        tgt = field_starts[fi + 1] if fi + 1 < len(fields) else done
        for s in field_ends[fi]:
            next_sep[s] = tgt

    S = len(states_allowed)
    E = max(1, max(len(e) for e in enum_lists))
    enum_tok = np.full((S, E), -1, dtype=np.int32)
    enum_next = np.full((S, E), -1, dtype=np.int32)
    for s, lst in enumerate(enum_lists):
        for j, (t, n) in enumerate(lst):
            enum_tok[s, j] = t
            enum_next[s, j] = n
    return SchemaFSM(
        fields=tuple(fields),
        vocab=vocab,
        sep_token=sep,
        allowed=np.stack(states_allowed),
        next_sep=np.asarray(next_sep, dtype=np.int32),
        next_tok=np.asarray(next_tok, dtype=np.int32),
        enum_tok=enum_tok,
        enum_next=enum_next,
        done_state=done,
        start_state=field_starts[0],
        field_of_state=field_of,
        copy_kind=np.asarray(copy_kind, dtype=np.int32),
        tok_flags=token_flags(strings, specials, vocab),
    )


def span_positions(max_body_tokens: int = 128) -> int:
    """Pointer tokens of the span format: one per prompt position (``body <ans>``)."""
    return max_body_tokens + 2


def build_span_fsm(tokenizer, vocab_tok: int, n_pos: int,
                   fields: Sequence[FieldSpec] = DEFAULT_FIELDS) -> SchemaFSM:
    """The span-pointer answer format (VERDICT r03 next #2a; sized by
    scripts/span_sim.py): the enum ``txn_type`` is written as in copy format (its
    trie, then ``<sep>``); every copied field is ONE pointer to its first body token
    and ONE to its last -- or ``<sep>`` for an empty value -- instead of its tokens
    one by one.  Pointer ``j`` is token id ``vocab_tok + j`` (ids past the tokenizer's
    vocabulary: the model's embedding row of pointer ``j`` is also added to the input
    of prompt position ``j``, so the model can name a position by "reading" it there).

    States per copied field: start (kind PTR_START | cap << 8 | class << 16: a pointer
    -> end, <sep> -> next field; only starts with at least one valid end are offered)
    and end (PTR_END | cap << 8 | class << 16: a pointer -> next field).  The
    vocabulary is rounded up to 128 (the lm_head / mask tiles)."""
    V = -(-(vocab_tok + n_pos) // 128) * 128
    strings = tokenizer.token_strings
    V_tok = len(strings)
    specials = [tokenizer.pad, tokenizer.bos, tokenizer.eos, tokenizer.sep, tokenizer.sms, tokenizer.ans]
    classes = _token_class_sets(strings, specials)
    sep = tokenizer.sep
    ptrs = np.zeros(V, dtype=bool)
    ptrs[vocab_tok:vocab_tok + n_pos] = True
    allowed: List[np.ndarray] = []
    next_sep: List[int] = []
    next_tok: List[int] = []
    enum_lists: List[List[Tuple[int, int]]] = []
    field_of: List[int] = []
    kinds: List[int] = []

    def new_state(mask: np.ndarray, fidx: int, kind: int = COPY_NONE) -> int:
        allowed.append(mask)
        next_sep.append(-1)
        next_tok.append(-1)
        enum_lists.append([])
        field_of.append(fidx)
        kinds.append(kind)
        return len(allowed) - 1

    starts: List[int] = []
    leaves: List[List[int]] = []  # per field: states whose <sep> / pointer leaves it
    for fi, f in enumerate(fields):
        if f.kind == "enum":
            enc = [tokenizer.encode(c) for c in f.choices]
            if max(len(e) for e in enc) > f.cap:
                raise ValueError(f"enum field {f.name!r}: a choice needs more than cap={f.cap} tokens")
            root = new_state(np.zeros(V, dtype=bool), fi)
            nodes: Dict[Tuple[int, ...], int] = {(): root}
            ends: List[int] = []
            for seq in enc:
                for d in range(len(seq)):
                    cur, key = nodes[tuple(seq[:d])], tuple(seq[:d + 1])
                    if key not in nodes:
                        nodes[key] = new_state(np.zeros(V, dtype=bool), fi)
                    allowed[cur][seq[d]] = True
                    if (seq[d], nodes[key]) not in enum_lists[cur]:
                        enum_lists[cur].append((seq[d], nodes[key]))
                    next_tok[cur] = -2
                allowed[nodes[tuple(seq)]][sep] = True
                ends.append(nodes[tuple(seq)])
            starts.append(root)
            leaves.append(ends)
        else:
            if not f.copy or f.cap > 64 or f.cap > 255:
                raise ValueError(f"span format: field {f.name!r} must be a copy field with cap <= 64")
            m = ptrs.copy()
            m[sep] = True
            cls = TOK_CLASS_BITS.get(f.kind, 0)
            # the start state carries the cap too: a start is offered only if it has an end
            a = new_state(m, fi, PTR_START | (f.cap << 8) | (cls << 16))
            b = new_state(ptrs.copy(), fi, PTR_END | (f.cap << 8) | (cls << 16))
            next_tok[a] = b
            starts.append(a)
            leaves.append([a, b])  # a: by <sep> (empty value); b: by its end pointer
    only_sep = np.zeros(V, dtype=bool)
    only_sep[sep] = True
    done = new_state(only_sep, len(fields))
    next_sep[done] = done
    for fi, f in enumerate(fields):
        tgt = starts[fi + 1] if fi + 1 < len(fields) else done
        if f.kind == "enum":
            for st in leaves[fi]:
                next_sep[st] = tgt
        else:
            a, b = leaves[fi]
            next_sep[a] = tgt
            next_tok[b] = tgt
    S = len(allowed)
    E = max(1, max(len(e) for e in enum_lists))
    enum_tok = np.full((S, E), -1, dtype=np.int32)
    enum_next = np.full((S, E), -1, dtype=np.int32)
    for st, lst in enumerate(enum_lists):
        for j, (t, nx) in enumerate(lst):
            enum_tok[st, j], enum_next[st, j] = t, nx
    return SchemaFSM(fields=tuple(fields), vocab=V, sep_token=sep, allowed=np.stack(allowed),
                     next_sep=np.asarray(next_sep, dtype=np.int32), next_tok=np.asarray(next_tok, dtype=np.int32),
                     enum_tok=enum_tok, enum_next=enum_next, done_state=done, start_state=starts[0],
                     field_of_state=field_of, copy_kind=np.asarray(kinds, dtype=np.int32),
                     tok_flags=token_flags(strings, specials, V, classes), ptr0=vocab_tok, n_pos=n_pos)
