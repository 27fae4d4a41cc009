"""Byte-level BPE tokenizer of the local extractor.

No pretrained tokenizer files exist on the box, so the extractor's tokenizer is
trained in-repo (``python -m smsgate_amd.models.tokenizer --train``) with the
Rust ``tokenizers`` library on the synthetic SMS corpus
(:mod:`smsgate_amd.utils.synth`) plus the system prompt, and committed as
``assets/extractor_tokenizer.json``.  Byte-level BPE never fails on unseen
text (Cyrillic, emoji…): unknown strings fall back to byte tokens.

Special tokens: ``<pad> <bos> <eos> <sep> <sms> <ans>``.  The prompt of one
extraction is ``<bos> EXTRACTOR_PROMPT <sms>`` (shared prefix, cached once on
the GPU) + ``body <ans>`` (per message); the answer is the nine field
values in schema order, each terminated by ``<sep>``.
"""
from __future__ import annotations

import functools
from pathlib import Path
from typing import List, Optional, Sequence, Tuple

__all__ = ["ExtractorTokenizer", "SPECIALS", "load_tokenizer", "train_tokenizer", "ASSET", "model_text"]

ASSET = Path(__file__).resolve().parent / "assets" / "extractor_tokenizer.json"
SPECIALS = ["<pad>", "<bos>", "<eos>", "<sep>", "<sms>", "<ans>"]
DEFAULT_VOCAB = 8192


# Pre-tokenizer: GPT-2's split, except that a NUMBER stays one pre-token -- digits joined
# by '.' / ':' (dates "06.05.25", times "14:23", decimals "52.00") or a thousands group
# ("1,842.74": ',' followed by exactly three digits).  Byte-level BPE never merges across
# pre-tokens, and GPT-2's split cut every number at each '.', ',' and ':' (a date + time
# was 8 tokens).  ',' before a non-3-digit group stays a separator ("BLVD 89,17.05.24"
# keeps the street number and the date apart), so every body value stays token-aligned.
# 8 192 merges: 49.2 -> 41.2 body tokens and 43.8 -> 35.7 answer tokens per purchase SMS.
# Currency symbols and card-mask star runs are pre-tokens of their own (never glued to
# neighbouring punctuation: "-£574.33", "BAL:$52.00", "CARD:**3736"), so a copied
# currency or masked card is token-aligned.
NUMBER_AWARE_SPLIT = (r"'s|'t|'re|'ve|'m|'ll|'d| ?\p{L}+| ?\d{1,3}(?:,\d{3})+(?:\.\d+)?| ?\d+(?:[.:]\d+)*"
                      r"| ?[$€£₽₾֏]| ?\*+| ?[^\s\p{L}\p{N}$€£₽₾֏*]+|\s+(?!\S)|\s+")


def train_tokenizer(path: Path = ASSET, vocab_size: int = DEFAULT_VOCAB, n_sms: int = 60000, seed: int = 1234):
    from tokenizers import Regex, Tokenizer, decoders, models, pre_tokenizers, trainers

    from ..parse.schema import EXTRACTOR_PROMPT, SYSTEM_INSTRUCTION
    from ..utils.synth import iter_corpus

    tok = Tokenizer(models.BPE())
    tok.pre_tokenizer = pre_tokenizers.Sequence([
        pre_tokenizers.Split(Regex(NUMBER_AWARE_SPLIT), behavior="isolated"),
        pre_tokenizers.ByteLevel(add_prefix_space=False, use_regex=False),
    ])
    tok.decoder = decoders.ByteLevel()
    trainer = trainers.BpeTrainer(
        vocab_size=vocab_size,
        special_tokens=SPECIALS,
        initial_alphabet=pre_tokenizers.ByteLevel.alphabet(),
        show_progress=False,
    )

    def corpus():
        for _ in range(50):
            yield SYSTEM_INSTRUCTION
            yield EXTRACTOR_PROMPT
        yield from (model_text(t) for t in iter_corpus(n_sms, seed))

    tok.train_from_iterator(corpus(), trainer=trainer)
    path.parent.mkdir(parents=True, exist_ok=True)
    tok.save(str(path))
    return tok


def model_text(text: str) -> str:
    """The text the extractor reads: bank bodies carry their line breaks as the literal
    XML entity ``&#10;`` (the reference's export), which byte-level BPE splits into three
    tokens (``&#`` ``10`` ``;``: the pre-tokenizer separates punctuation from digits) --
    15 of the ~55 tokens of an account-format SMS.  The model sees one ``\n`` token
    instead.  No extracted value spans a line break, so copied values are unchanged."""
    return text.replace("&#10;", "\n") if "&#" in text else text


class ExtractorTokenizer:
    def __init__(self, path: Path = ASSET) -> None:
        from tokenizers import Tokenizer

        if not Path(path).exists():
            train_tokenizer(Path(path))
        self.tk = Tokenizer.from_file(str(path))
        self.vocab_size = self.tk.get_vocab_size()
        ids = {s: self.tk.token_to_id(s) for s in SPECIALS}
        self.pad, self.bos, self.eos, self.sep, self.sms, self.ans = (ids[s] for s in SPECIALS)

    def encode(self, text: str) -> List[int]:
        return self.tk.encode(model_text(text), add_special_tokens=False).ids

    def encode_batch(self, texts: Sequence[str]) -> List[List[int]]:
        # the offset-free batch encoder: same ids, ~25 % less work (offsets are only
        # needed for training targets, encode_offsets)
        return [e.ids for e in self.tk.encode_batch_fast([model_text(t) for t in texts], add_special_tokens=False)]

    def encode_offsets(self, texts: Sequence[str]) -> List[Tuple[List[int], List[Tuple[int, int]]]]:
        """Ids plus each token's ``(start, end)`` character span in its MODEL text
        (:func:`model_text`; a token that carries a leading blank covers it)."""
        return [(e.ids, e.offsets) for e in self.tk.encode_batch([model_text(t) for t in texts],
                                                                  add_special_tokens=False)]

    def value_span_ids(self, value: str, body: str, ids: Sequence[int],
                       offsets: Sequence[Tuple[int, int]]) -> List[int]:
        """How the extractor writes a field value: the body's own tokens covering
        it when the value is a token-aligned substring of the body (decoding them
        and stripping blanks gives back ``value``), else ``encode(value)``.

        Copying the body's tokens verbatim is what the model is trained to do, so
        a value costs as many decode steps as it has in the body, and the body is
        an exact draft for speculative decoding (:mod:`smsgate_amd.serving.draft`)."""
        if not value:
            return []
        sp = self.value_span(value, body, ids, offsets)
        return list(ids[sp[0]:sp[1] + 1]) if sp is not None else self.encode(value)

    def value_span(self, value: str, body: str, ids: Sequence[int],
                   offsets: Sequence[Tuple[int, int]]) -> Optional[Tuple[int, int]]:
        """``(first, last)`` body token index of the first word-aligned occurrence of
        ``value`` whose tokens decode back to it (:meth:`value_span_ids`; the span
        format points at these two positions), or None."""
        body, value = model_text(body), model_text(value)  # the offsets index the model text
        sp = self._value_span(value, body, ids, offsets, strict=True)
        # a value glued to a word of the other kind ("52.00" in "USD52.00", "1234" in
        # "x1234"): only when it occurs nowhere at a full word boundary, so a number inside
        # a merchant name ("AB52") never shadows the real amount
        return sp if sp is not None else self._value_span(value, body, ids, offsets, strict=False)

    def _value_span(self, value: str, body: str, ids, offsets, strict: bool) -> Optional[Tuple[int, int]]:
        def glued(x: str, y: str) -> bool:
            if strict:
                return x.isalnum() and y.isalnum()
            return (x.isalpha() and y.isalpha()) or (x.isdigit() and y.isdigit())

        start = 0
        while True:
            a = body.find(value, start)
            if a < 0:
                return None
            z = a + len(value)
            # an occurrence inside a longer word is not the value ("AM" in "AMERIABANK"
            # vs the city ", AM&#10;"): values are copied at word boundaries (the copy
            # constraint, serving/fsm.py, only lets a value start and end there)
            if (a > 0 and glued(body[a - 1], value[0])) or (z < len(body) and glued(value[-1], body[z])):
                start = a + 1
                continue
            k0 = next((k for k, (s, e) in enumerate(offsets) if s <= a < e), None)
            # the LAST token ending at z: a character split over several byte-level
            # tokens (Cyrillic, symbols) gives each piece the character's whole span
            k1 = max((k for k, (s, e) in enumerate(offsets) if e == z), default=None)
            if k0 is not None and k1 is not None and k1 >= k0 and body[offsets[k0][0]:a].strip() == "":
                if self.decode(list(ids[k0:k1 + 1])).strip() == value:
                    return k0, k1
            start = a + 1

    def decode(self, ids: Sequence[int]) -> str:
        return self.tk.decode(list(ids), skip_special_tokens=True)

    @functools.cached_property
    def token_bytes(self) -> List[bytes]:
        """The raw bytes of every id (specials -> ``b""``): byte-level BPE tokens are
        byte strings, so a value decodes as ``b"".join(...).decode("utf-8", "replace")``
        -- identical to :meth:`decode` (tests/test_families.py pins it) without a
        round trip through the library per value."""
        u2b = {c: b for b, c in _bytes_to_unicode().items()}
        out = [b""] * self.vocab_size
        for s, i in self.tk.get_vocab().items():
            if s not in SPECIALS and i < self.vocab_size:
                out[i] = bytes(u2b[c] for c in s)
        return out

    def decode_fields(self, seqs: Sequence[Sequence[int]], nfields: int) -> List[List[str]]:
        """Answer token sequences -> ``nfields`` stripped strings each (split at
        ``<sep>``; a missing field is ``""``; tokens after the last field are dropped)."""
        tb = self.token_bytes
        sep = self.sep
        out: List[List[str]] = []
        for toks in seqs:
            vals: List[str] = []
            cur: List[bytes] = []
            for t in toks:
                if t == sep:
                    vals.append(b"".join(cur).decode("utf-8", "replace").strip())
                    if len(vals) == nfields:
                        break
                    cur = []
                else:
                    cur.append(tb[t])
            else:
                if len(vals) < nfields:
                    vals.append(b"".join(cur).decode("utf-8", "replace").strip())
            vals += [""] * (nfields - len(vals))
            out.append(vals)
        return out

    def decode_batch(self, seqs: Sequence[Sequence[int]]) -> List[str]:
        return self.tk.decode_batch([list(s) for s in seqs], skip_special_tokens=True)

    @functools.cached_property
    def token_strings(self) -> List[str]:
        """Decoded text of every id (specials → their literal)."""
        out = []
        for i in range(self.vocab_size):
            s = self.tk.id_to_token(i)
            out.append(s if s in SPECIALS else self.tk.decode([i], skip_special_tokens=False))
        return out

    def prefix_ids(self, system: str) -> List[int]:
        """``<bos> system <sms>``: the shared prefix ends with the message marker, so
        it is computed once instead of once per message."""
        return [self.bos] + self.encode(system) + [self.sms]

    truncated = 0  # bodies cut to max_body tokens (also the llm_prompt_truncated_total counter)

    def message_ids(self, bodies: Sequence[str], max_body: int) -> List[List[int]]:
        """``body <ans>`` ids (the ``<sms>`` marker ends the shared prefix,
        :meth:`prefix_ids`).  A body longer than ``max_body`` tokens keeps
        its first ``max_body`` tokens; every such cut is counted (the extractor
        never sees the tail, where balances often are), never silent."""
        enc = self.encode_batch(bodies)
        cut = sum(1 for e in enc if len(e) > max_body)
        if cut:
            self.truncated += cut
            from ..obs.metrics import LLM_TRUNCATED

            LLM_TRUNCATED.inc(cut)
        return [e[:max_body] + [self.ans] for e in enc]


def _bytes_to_unicode() -> dict:
    """GPT-2's byte <-> printable-character table (the ByteLevel pre-tokenizer's alphabet)."""
    bs = list(range(ord("!"), ord("~") + 1)) + list(range(ord("¡"), ord("¬") + 1)) + list(range(ord("®"), ord("ÿ") + 1))
    cs = bs[:]
    n = 0
    for b in range(256):
        if b not in bs:
            bs.append(b)
            cs.append(256 + n)
            n += 1
    return dict(zip(bs, (chr(c) for c in cs)))


@functools.lru_cache(maxsize=4)
def load_tokenizer(path: str = str(ASSET)) -> ExtractorTokenizer:
    return ExtractorTokenizer(Path(path))


if __name__ == "__main__":
    import sys
    import time

    if "--train" in sys.argv:
        t0 = time.time()
        tk = train_tokenizer()
        print(f"trained vocab={tk.get_vocab_size()} in {time.time() - t0:.1f}s -> {ASSET}")
    t = load_tokenizer()
    from ..utils.synth import reference_cases

    for b in reference_cases():
        ids = t.encode(b)
        print(len(b), "chars ->", len(ids), "tokens")
